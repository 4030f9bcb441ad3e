package lgbt.princess.reservoir.gpu

import java.lang.ref.{PhantomReference, ReferenceQueue}
import java.util.Arrays
import java.util.concurrent.ConcurrentHashMap

import scala.collection.immutable.ArraySeq

import lgbt.princess.reservoir.Sampler

/** JNI natives of bindings/jni/reservoir_jni.c, for the reference's CI JDKs 8/11/15 (build.sbt:37-42).
  * No native call holds a JVM array pinned while the engine may wait: keys are copied with
  * Get<Type>ArrayRegion straight into the engine's pinned staging, results come back through a
  * native buffer and Set<Type>ArrayRegion.
  * A session is a native rsv_jvm (bindings/jvm/rsv_jvm.h) held as a Long. */
private[reservoir] object Jni {
  System.loadLibrary("reservoir_jni")

  @native def create(
      kind: Int,
      k: Int,
      keyWidth: Int,
      reusable: Boolean,
      engine: Int,
      hashKind: Int,
      order: Int,
      seed: Long,
      streamId: Long,
      device: Int,
  ): Long
  @native def sampleLong(session: Long, key: Long, hash: Long): Unit
  @native def sampleInt(session: Long, key: Int, hash: Long): Unit
  @native def sampleLongs(session: Long, keys: Array[Long], hashes: Array[Long], n: Int): Unit
  @native def sampleInts(session: Long, keys: Array[Int], hashes: Array[Long], n: Int): Unit
  @native def resultLongs(session: Long, out: Array[Long]): Int
  @native def resultInts(session: Long, out: Array[Int]): Int
  @native def isOpen(session: Long): Boolean
  @native def destroy(session: Long): Unit
  @native def stageAcquire(session: Long): java.nio.ByteBuffer
  @native def stageCommit(session: Long, n: Long): Unit
  @native def sampleIndexed(session: Long, n: Long, offsets: Array[Long]): Unit
  @native def fillLongs(session: Long, keys: Array[Long]): Unit
  @native def fillInts(session: Long, keys: Array[Int]): Unit
  // byte keys (UUID): key_width / 8 Longs per key, n counts keys
  @native def sampleWords(session: Long, words: Array[Long], hashes: Array[Long], n: Int): Unit
  @native def resultWords(session: Long, out: Array[Long]): Int
  @native def fillWords(session: Long, words: Array[Long]): Unit
  @native def abortIndexed(session: Long): Unit
  @native def commitIndexed(session: Long): Unit
}

/** One native session (a malloc'd rsv_jvm, reservoir_jni.c) released exactly once: by a single-use
  * `result()`, or by [[JniCleaner]] once its sampler is unreachable. */
private[gpu] final class JniSession(initial: Long) {
  @volatile private[this] var ptr = initial
  def get: Long = ptr
  def release(): Unit = synchronized {
    if (ptr != 0L) {
      Jni.destroy(ptr)
      ptr = 0L
    }
  }
}

/** JDK 8 has no java.lang.ref.Cleaner and `finalize()` is deprecated since JDK 9 (an error under
  * -Xlint -Werror on the reference's newer CI JDKs): a phantom reference per sampler on one queue,
  * drained by a daemon thread that releases the session.  The reference holds the session, never
  * the sampler, so the sampler can become unreachable. */
private[gpu] object JniCleaner {
  private final class Ref(owner: AnyRef, val session: JniSession, q: ReferenceQueue[AnyRef])
      extends PhantomReference[AnyRef](owner, q)

  private[this] val queue = new ReferenceQueue[AnyRef]
  private[this] val live  = ConcurrentHashMap.newKeySet[Ref]() // the Refs themselves must stay reachable

  private[this] val thread = {
    val t = new Thread(new Runnable {
      def run(): Unit =
        while (true) {
          val r = queue.remove().asInstanceOf[Ref]
          live.remove(r)
          r.session.release()
        }
    }, "reservoir-jni-cleaner")
    t.setDaemon(true)
    t.start()
    t
  }

  def register(owner: AnyRef, session: JniSession): Unit = {
    live.add(new Ref(owner, session, queue))
    ()
  }
}

/** A GPU-backed `Sampler[A, B]` over JNI, B = Long, Int or UUID (any other B: [[ObjectSampler]]): keys are buffered in a JVM array and
  * handed over 65536 at a time (one JNI call per batch, none per element); the native session copies
  * them into the engine's pinned staging buffer.  Lifecycle as FfmSampler: `isOpen` tracked here, the
  * single-use `result()` destroys the session at once. */
private[reservoir] final class JniSampler[A, B](
    kind: Int,
    maxSampleSize: Int,
    reusable: Boolean,
    keys: KeyKind[B],
    hashKind: Int,
    engine: Int,
    seed: Long,
)(map: A => B, hash: B => Long)
    extends Sampler[A, B] {
  private[this] final val Batch = 65536
  private[this] val isLong      = keys.width == 8
  private[this] val isUuid      = keys eq KeyKind.UuidKey
  private[this] val precomputed = kind == Abi.KindDistinct && hashKind == Abi.HashPrecomputed
  private[this] val session =
    new JniSession(Jni.create(kind, maxSampleSize, keys.width, reusable, engine, hashKind, Abi.OrderAuto, seed, 0L, -1))
  JniCleaner.register(this, session)
  private[this] val longs  = if (isLong) new Array[Long](Batch) else if (isUuid) new Array[Long](2 * Batch) else null
  private[this] val ints   = if (isLong || isUuid) null else new Array[Int](Batch)
  private[this] val hashes = if (precomputed) new Array[Long](Batch) else null
  private[this] var n      = 0
  private[this] var open   = true
  // Every native call passes the raw session pointer only, so the JIT may consider `this` dead
  // during the call and let JniCleaner release the session under it.  A volatile store to this
  // field after each call keeps `this` reachable until the call has returned (JDK 8 has no
  // Reference.reachabilityFence).
  @volatile private[this] var fence = 0

  private[this] def flush(): Unit =
    if (n > 0) {
      if (isUuid) Jni.sampleWords(session.get, longs, hashes, n)
      else if (isLong) Jni.sampleLongs(session.get, longs, hashes, n)
      else Jni.sampleInts(session.get, ints, hashes, n)
      n = 0
      fence = 1
    }

  def sample(element: A): Unit = {
    if (!open) throw new IllegalStateException(Abi.ClosedMessage)
    val b = map(element)
    if (isUuid) {
      val u = b.asInstanceOf[java.util.UUID]
      longs(2 * n) = u.getMostSignificantBits
      longs(2 * n + 1) = u.getLeastSignificantBits
    } else if (isLong) longs(n) = b.asInstanceOf[Long]
    else ints(n) = b.asInstanceOf[Int]
    if (precomputed) hashes(n) = hash(b)
    n += 1
    if (n == Batch) flush()
  }

  /** sampleAll over a known-size IndexedSeq (Sampler.scala:289-312 -> sampleIndexed :261-273): the
    * engine samples the indices alone, and `map` runs only on the elements that end up holding a
    * slot -- no key crosses JNI or PCIe for the rest (the reference reads ~k ln(n/k) of them).
    * Distinct samplers keep the trait's per-element default (Sampler.scala:50). */
  override def sampleAll(elements: IterableOnce[A]): Unit = elements match {
    case seq: collection.IndexedSeq[A @unchecked] if kind == Abi.KindElements && seq.knownSize > 0 =>
      if (!open) throw new IllegalStateException(Abi.ClosedMessage)
      flush()
      val offsets = new Array[Long](maxSampleSize)
      Jni.sampleIndexed(session.get, seq.length.toLong, offsets)
      // a throwing `map` drops the batch (the sampler stays usable) and propagates, as the
      // reference's sampleIndexed propagates it; the fill downcall runs outside the try, as in
      // FfmSampler (a failed fill is the engine's error, not the user's)
      val longKeys = if (isUuid) new Array[Long](2 * maxSampleSize) else if (isLong) new Array[Long](maxSampleSize) else null
      val intKeys  = if (longKeys == null) new Array[Int](maxSampleSize) else null
      try {
        var j = 0
        while (j < maxSampleSize) {
          val o = offsets(j)
          if (o >= 0) {
            val b = map(seq(o.toInt))
            if (isUuid) {
              val u = b.asInstanceOf[java.util.UUID]
              longKeys(2 * j) = u.getMostSignificantBits
              longKeys(2 * j + 1) = u.getLeastSignificantBits
            } else if (isLong) longKeys(j) = b.asInstanceOf[Long]
            else intKeys(j) = b.asInstanceOf[Int]
          }
          j += 1
        }
      } catch {
        case t: Throwable =>
          try Jni.abortIndexed(session.get)
          catch { case e: Throwable => t.addSuppressed(e) }
          fence = 1
          throw t
      }
      if (isUuid) Jni.fillWords(session.get, longKeys)
      else if (isLong) Jni.fillLongs(session.get, longKeys)
      else Jni.fillInts(session.get, intKeys)
      fence = 1
    case _ => super.sampleAll(elements)
  }

  def result(): IndexedSeq[B] = {
    if (!open) throw new IllegalStateException(Abi.ClosedMessage)
    flush()
    val res =
      if (isUuid) {
        val out = new Array[Long](2 * maxSampleSize)
        val m   = Jni.resultWords(session.get, out)
        ArraySeq.unsafeWrapArray(Array.tabulate(m)(i => new java.util.UUID(out(2 * i), out(2 * i + 1))))
      } else if (isLong) {
        val out = new Array[Long](maxSampleSize)
        val m   = Jni.resultLongs(session.get, out)
        ArraySeq.unsafeWrapArray(if (m == out.length) out else Arrays.copyOf(out, m))
      } else {
        val out = new Array[Int](maxSampleSize)
        val m   = Jni.resultInts(session.get, out)
        ArraySeq.unsafeWrapArray(if (m == out.length) out else Arrays.copyOf(out, m))
      }
    fence = 1
    if (!reusable) { // the native side destroyed the handle inside result(); free the session now
      open = false
      session.release()
    }
    res.asInstanceOf[IndexedSeq[B]]
  }

  def isOpen: Boolean = open
}

/** [[IndexOps]] over JNI: an ELEMENTS session whose slots the engine fills by index only
  * (rsv_commit_indexed); the B values live in the [[ObjectSampler]]. */
private[reservoir] final class JniIndexOps(k: Int, reusable: Boolean, engine: Int, seed: Long) extends IndexOps {
  private[this] val session =
    new JniSession(Jni.create(Abi.KindElements, k, 8, reusable, engine, Abi.HashDefault, Abi.OrderAuto, seed, 0L, -1))
  JniCleaner.register(this, session)
  @volatile private[this] var fence = 0 // keeps `this` reachable across each native call (JniSampler)

  def sampleIndexed(n: Long, offsets: Array[Long]): Unit = { Jni.sampleIndexed(session.get, n, offsets); fence = 1 }
  def commitIndexed(): Unit                              = { Jni.commitIndexed(session.get); fence = 1 }
  def abortIndexed(): Unit                               = { Jni.abortIndexed(session.get); fence = 1 }
  def release(): Unit                                    = session.release()
}
