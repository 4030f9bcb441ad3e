package lgbt.princess.reservoir.gpu

import scala.collection.immutable.ArraySeq
import scala.reflect.ClassTag

import lgbt.princess.reservoir.Sampler

/** The downcalls an [[ObjectSampler]] makes: index-only batches (include/reservoir_hip.h
  * rsv_sample_indexed / rsv_commit_indexed / rsv_abort_indexed) and the handle's release.  The JNI
  * binding implements it over `Jni` (JniSampler.scala), the FFM binding over its downcall handles
  * (FfmSampler.scala). */
private[reservoir] trait IndexOps {

  /** the next n elements by index: offsets(j) = the batch offset of slot j's new holder, or -1 */
  def sampleIndexed(n: Long, offsets: Array[Long]): Unit

  /** accept the pending batch; the elements stay on the JVM */
  def commitIndexed(): Unit

  /** drop the pending batch (a `map` threw) */
  def abortIndexed(): Unit

  /** destroy the handle (a single-use result(), or the cleaner) */
  def release(): Unit
}

/** A GPU-backed `Sampler[A, B]` for ANY `B` (a case class, a String, any object: Sampler.scala:128-136
  * takes every `B` with a ClassTag), where `B` has no fixed-width key the engine could store.
  *
  * The engine still decides which element each slot holds -- from the element indices alone, with
  * the same draws (philox_r) or the same java.util.Random Algorithm L events (java_l) as a keyed
  * sampler -- and this class keeps the k-slot array of `B` references itself, as RandomElements
  * keeps `samples` (Sampler.scala:200-202):
  *   - `sampleAll` over a known-size IndexedSeq: one index-only batch (rsv_sample_indexed), then
  *     `map` runs only on the elements that now hold a slot (sampleIndexed reads only those,
  *     Sampler.scala:261-273) and they go straight into the slot array; no element crosses JNI or
  *     PCIe, and a throwing `map` drops the batch (rsv_abort_indexed) and propagates;
  *   - `sample` (and `sampleAll` over anything else): `map` applied per element as the keyed
  *     samplers do (Sampler.scala:115-116 allows the extra calls), the mapped elements buffered
  *     here 65536 at a time; a full buffer is sampled by index and its winners copied over.
  * `result()` wraps the slot array like resultImpl (Sampler.scala:318-331); a reusable sampler
  * copies it before its next sample once a result aliases it, like MultiResultRandomElements.
  *
  * tests/cpp/test_ffm_sequence.cpp (ObjectMirror) replays this class's downcalls on the GPU. */
private[reservoir] final class ObjectSampler[A, B: ClassTag](maxSampleSize: Int, reusable: Boolean, ops: IndexOps)(
    map: A => B
) extends Sampler[A, B] {
  private[this] final val Batch = 65536
  private[this] var slots: Array[B] = new Array[B](math.min(16, maxSampleSize))
  private[this] var aliased         = false // a reusable result() wraps `slots`
  private[this] val pending         = new Array[AnyRef](Batch) // mapped elements of sample(), boxed
  private[this] var n               = 0
  private[this] var count           = 0L
  private[this] var offsets: Array[Long] = _
  private[this] var open            = true

  /** room for slot j: doubling up to maxSampleSize (the fill phase writes slots in order) */
  private[this] def ensureSize(j: Int): Unit =
    if (slots.length <= j) {
      val len  = slots.length
      val grow = if (len >= (Int.MaxValue >> 1)) maxSampleSize else math.min(maxSampleSize, len << 1)
      val next = new Array[B](math.max(grow, j + 1))
      System.arraycopy(slots, 0, next, 0, len)
      slots = next
    }

  private[this] def unalias(): Unit =
    if (aliased) {
      slots = slots.clone()
      aliased = false
    }

  private[this] def offsetArray(): Array[Long] = {
    if (offsets == null) offsets = new Array[Long](maxSampleSize)
    offsets
  }

  /** the buffered, already mapped elements as one index-only batch */
  private[this] def flush(): Unit =
    if (n > 0) {
      val o = offsetArray()
      ops.sampleIndexed(n.toLong, o)
      ops.commitIndexed() // nothing left to map: the batch is final
      unalias()
      var j = 0
      while (j < maxSampleSize) {
        val x = o(j)
        if (x >= 0) {
          ensureSize(j)
          slots(j) = pending(x.toInt).asInstanceOf[B]
        }
        j += 1
      }
      java.util.Arrays.fill(pending, 0, n, null) // let the elements go
      count += n
      n = 0
    }

  def sample(element: A): Unit = {
    if (!open) throw new IllegalStateException(Abi.ClosedMessage)
    pending(n) = map(element).asInstanceOf[AnyRef]
    n += 1
    if (n == Batch) flush()
  }

  override def sampleAll(elements: IterableOnce[A]): Unit = elements match {
    case seq: collection.IndexedSeq[A @unchecked] if seq.knownSize > 0 =>
      if (!open) throw new IllegalStateException(Abi.ClosedMessage)
      flush()
      val len = seq.length
      val o   = offsetArray()
      ops.sampleIndexed(len.toLong, o)
      // map the new holders first; the slots change only once every one of them has been mapped
      var changed = 0
      var j       = 0
      while (j < maxSampleSize) { if (o(j) >= 0) changed += 1; j += 1 }
      val js   = new Array[Int](changed)
      val vals = new Array[B](changed)
      var c    = 0
      try {
        j = 0
        while (j < maxSampleSize) {
          val x = o(j)
          if (x >= 0) {
            js(c) = j
            vals(c) = map(seq(x.toInt))
            c += 1
          }
          j += 1
        }
      } catch {
        case t: Throwable => // drop the batch, keep the sampler usable, propagate (sampleIndexed does)
          try ops.abortIndexed()
          catch { case e: Throwable => t.addSuppressed(e) }
          throw t
      }
      ops.commitIndexed()
      unalias()
      c = 0
      while (c < changed) {
        ensureSize(js(c))
        slots(js(c)) = vals(c)
        c += 1
      }
      count += len
    case _ => super.sampleAll(elements)
  }

  def result(): IndexedSeq[B] = {
    if (!open) throw new IllegalStateException(Abi.ClosedMessage)
    flush()
    val m = math.min(count, maxSampleSize.toLong).toInt
    val arr =
      if (m == slots.length) slots
      else {
        val res = new Array[B](m)
        System.arraycopy(slots, 0, res, 0, m)
        res
      }
    if (!reusable) {
      open = false
      slots = null
      ops.release()
    } else if (arr eq slots) aliased = true
    ArraySeq.unsafeWrapArray(arr)
  }

  def isOpen: Boolean = open
}
