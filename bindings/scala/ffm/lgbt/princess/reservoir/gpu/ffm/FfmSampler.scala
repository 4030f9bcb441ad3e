package lgbt.princess.reservoir.gpu.ffm

// JDK 22+ only: the separate sbt module reservoir-gpu-ffm (INTEGRATION.md), loaded by gpu.Backend
// through Class.forName, so the core module never links java.lang.foreign.

import java.lang.foreign.{Arena, FunctionDescriptor, Linker, MemoryLayout, MemorySegment, StructLayout, SymbolLookup}
import java.lang.foreign.ValueLayout.{ADDRESS, JAVA_INT, JAVA_LONG}
import java.lang.invoke.MethodHandle
import java.lang.ref.Cleaner

import scala.collection.immutable.ArraySeq
import scala.reflect.ClassTag

import lgbt.princess.reservoir.Sampler
import lgbt.princess.reservoir.gpu.{Abi, IndexOps, KeyKind, ObjectSampler, SamplerFactory}

/** Panama FFM downcall handles of libreservoir_hip.so (JDK 22+, run with --enable-native-access).
  * Names carry an `rsv` prefix so nothing here shadows a Sampler member (e.g. `isOpen`). */
private[reservoir] object Native {
  private val linker = Linker.nativeLinker()
  private val lib =
    SymbolLookup.libraryLookup(System.getProperty("reservoir.hip.lib", "libreservoir_hip.so"), Arena.global())
  private def downcall(name: String, fd: FunctionDescriptor): MethodHandle =
    linker.downcallHandle(lib.find(name).orElseThrow(), fd)

  /** struct rsv_config (include/reservoir_hip.h): 10 x int32 then 2 x uint64 = 56 bytes. */
  val Config: StructLayout = MemoryLayout.structLayout(
    JAVA_INT.withName("struct_size"),
    JAVA_INT.withName("kind"),
    JAVA_INT.withName("max_sample_size"),
    JAVA_INT.withName("key_width"),
    JAVA_INT.withName("reusable"),
    JAVA_INT.withName("pre_allocate"),
    JAVA_INT.withName("engine"),
    JAVA_INT.withName("hash_kind"),
    JAVA_INT.withName("device"),
    JAVA_INT.withName("distinct_order"),
    JAVA_LONG.withName("seed"),
    JAVA_LONG.withName("stream_id"),
  )

  val rsvConfigInit: MethodHandle   = downcall("rsv_config_init", FunctionDescriptor.of(JAVA_INT, ADDRESS))
  val rsvCreate: MethodHandle       = downcall("rsv_create", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS))
  val rsvDestroy: MethodHandle      = downcall("rsv_destroy", FunctionDescriptor.ofVoid(ADDRESS))
  val rsvStageAcquire: MethodHandle =
    downcall("rsv_stage_acquire", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, ADDRESS))
  val rsvStageCommit: MethodHandle = downcall("rsv_stage_commit", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG))
  val rsvResult: MethodHandle =
    downcall("rsv_result", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS))
  val rsvLastError: MethodHandle = downcall("rsv_last_error", FunctionDescriptor.of(ADDRESS))
  val rsvSampleIndexed: MethodHandle =
    downcall("rsv_sample_indexed", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS))
  val rsvFillSlots: MethodHandle = downcall("rsv_fill_slots", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS))
  val rsvAbortIndexed: MethodHandle = downcall("rsv_abort_indexed", FunctionDescriptor.of(JAVA_INT, ADDRESS))
  val rsvCommitIndexed: MethodHandle = downcall("rsv_commit_indexed", FunctionDescriptor.of(JAVA_INT, ADDRESS))

  val cleaner: Cleaner = Cleaner.create()

  /** rsv_status -> the reference's exceptions (Abi.exception). */
  def check(status: Int): Unit =
    if (status != Abi.Ok) {
      val msg = rsvLastError.invoke().asInstanceOf[MemorySegment].reinterpret(Long.MaxValue).getString(0L)
      throw Abi.exception(status, msg)
    }
}

/** A GPU-backed `Sampler[A, B]` over Panama FFM, B = Long, Int or UUID ([mostSigBits | leastSigBits]).  `map` writes each key straight into
  * the engine's pinned staging buffer (rsv_stage_acquire / rsv_stage_commit: zero copy, double
  * buffered, flushed to the GPU asynchronously): one downcall per ~1 Mi keys and none per element.
  * `isOpen` is tracked here (no downcall); a single-use `result()` destroys the handle at once and
  * nothing touches it afterwards (Sampler.scala:182-194, :345-350).
  *
  * tests/cpp/test_ffm_sequence.cpp (FfmMirror) replays this class's calls, statement for
  * statement, on the GPU. */
private[reservoir] final class FfmSampler[A, B](
    kind: Int,
    maxSampleSize: Int,
    reusable: Boolean,
    keys: KeyKind[B],
    hashKind: Int,
    engine: Int,
    seed: Long,
)(map: A => B, hash: B => Long)
    extends Sampler[A, B] {
  import Native._

  private[this] val arena       = Arena.ofShared() // akka may call from different (sequential) threads
  private[this] val isLong      = keys.width == 8
  private[this] val isUuid      = keys eq KeyKind.UuidKey
  private[this] val precomputed = kind == Abi.KindDistinct && hashKind == Abi.HashPrecomputed
  private[this] val handle: MemorySegment = {
    // UUID keys travel as 2 Longs each in one segment / JVM array (result, sampleAll): as rsv_jvm_create
    if (isUuid && 2L * maxSampleSize > Int.MaxValue)
      throw new IllegalArgumentException("requirement failed: maxSampleSize * key words exceeds the JVM array limit")
    val cfg = arena.allocate(Config)
    check(rsvConfigInit.invoke(cfg).asInstanceOf[Int])
    cfg.set(JAVA_INT, 4L, kind)
    cfg.set(JAVA_INT, 8L, maxSampleSize)
    cfg.set(JAVA_INT, 12L, keys.width)
    cfg.set(JAVA_INT, 16L, if (reusable) 1 else 0)
    cfg.set(JAVA_INT, 24L, engine)
    cfg.set(JAVA_INT, 28L, hashKind)
    cfg.set(JAVA_LONG, 40L, seed)
    val out = arena.allocate(ADDRESS)
    check(rsvCreate.invoke(cfg, out).asInstanceOf[Int])
    out.get(ADDRESS, 0L)
  }
  // a reusable sampler is released when it becomes unreachable; a single-use one by result()
  private[this] val cleanable = {
    val h = handle
    val a = arena
    cleaner.register(this, () => { rsvDestroy.invoke(h); a.close() })
  }
  private[this] val keysOut   = arena.allocate(ADDRESS)
  private[this] val hashesOut = arena.allocate(ADDRESS)
  private[this] val capOut    = arena.allocate(JAVA_LONG)

  private[this] var open                    = true
  private[this] var stage: MemorySegment     = MemorySegment.NULL // engine-owned pinned memory
  private[this] var stageHash: MemorySegment = MemorySegment.NULL
  private[this] var cap                     = 0L
  private[this] var filled                  = 0L

  private[this] def nextStage(): Unit = {
    if (filled > 0) {
      val f = filled
      filled = 0
      cap = 0
      check(rsvStageCommit.invoke(handle, f).asInstanceOf[Int])
    }
    check(
      rsvStageAcquire.invoke(handle, keysOut, if (precomputed) hashesOut else MemorySegment.NULL, capOut).asInstanceOf[Int]
    )
    cap = capOut.get(JAVA_LONG, 0L)
    stage = keysOut.get(ADDRESS, 0L).reinterpret(cap * keys.width)
    if (precomputed) stageHash = hashesOut.get(ADDRESS, 0L).reinterpret(cap * 8)
  }

  /** a UUID key at index i of a key segment: [mostSigBits | leastSigBits] */
  private[this] def put(seg: MemorySegment, i: Long, b: B): Unit = {
    val u = b.asInstanceOf[java.util.UUID]
    seg.setAtIndex(JAVA_LONG, 2 * i, u.getMostSignificantBits)
    seg.setAtIndex(JAVA_LONG, 2 * i + 1, u.getLeastSignificantBits)
  }

  def sample(element: A): Unit = {
    if (!open) throw new IllegalStateException(Abi.ClosedMessage)
    if (filled == cap) nextStage()
    val b = map(element)
    if (isUuid) put(stage, filled, b)
    else if (isLong) stage.setAtIndex(JAVA_LONG, filled, b.asInstanceOf[Long])
    else stage.setAtIndex(JAVA_INT, filled, b.asInstanceOf[Int])
    if (precomputed) stageHash.setAtIndex(JAVA_LONG, filled, hash(b))
    filled += 1
  }

  /** sampleAll over a known-size IndexedSeq (Sampler.scala:289-312 -> sampleIndexed :261-273): the
    * engine samples the indices alone (rsv_sample_indexed) and `map` runs only on the elements now
    * holding a slot, whose keys go back in one downcall (rsv_fill_slots).  Distinct samplers keep
    * the trait's per-element default (Sampler.scala:50). */
  override def sampleAll(elements: IterableOnce[A]): Unit = elements match {
    case seq: collection.IndexedSeq[A @unchecked] if kind == Abi.KindElements && seq.knownSize > 0 =>
      if (!open) throw new IllegalStateException(Abi.ClosedMessage)
      if (filled > 0) { // the staged keys come first in index order
        val f = filled
        filled = 0
        check(rsvStageCommit.invoke(handle, f).asInstanceOf[Int])
      }
      cap = 0
      val tmp = Arena.ofConfined()
      try {
        val offsets = tmp.allocate(8L * maxSampleSize, 8L)
        check(rsvSampleIndexed.invoke(handle, seq.length.toLong, offsets).asInstanceOf[Int])
        val ks = tmp.allocate(keys.width.toLong * maxSampleSize, 8L)
        var j  = 0
        try {
          while (j < maxSampleSize) {
            val o = offsets.getAtIndex(JAVA_LONG, j.toLong)
            if (o >= 0) {
              val b = map(seq(o.toInt))
              if (isUuid) put(ks, j.toLong, b)
              else if (isLong) ks.setAtIndex(JAVA_LONG, j.toLong, b.asInstanceOf[Long])
              else ks.setAtIndex(JAVA_INT, j.toLong, b.asInstanceOf[Int])
            }
            j += 1
          }
        } catch { // `map` threw: drop the batch, keep the sampler usable, propagate (sampleIndexed does)
          case t: Throwable =>
            try check(rsvAbortIndexed.invoke(handle).asInstanceOf[Int])
            catch { case e: Throwable => t.addSuppressed(e) }
            throw t
        }
        check(rsvFillSlots.invoke(handle, ks).asInstanceOf[Int])
      } finally tmp.close()
    case _ => super.sampleAll(elements)
  }

  def result(): IndexedSeq[B] = {
    if (!open) throw new IllegalStateException(Abi.ClosedMessage)
    if (filled > 0) {
      val f = filled
      filled = 0
      check(rsvStageCommit.invoke(handle, f).asInstanceOf[Int])
    }
    cap = 0 // the staging pointers are valid only until the next call on the handle
    val tmp = Arena.ofConfined()
    val res =
      try {
        val out = tmp.allocate(keys.width.toLong * maxSampleSize, 8L)
        val n   = tmp.allocate(JAVA_LONG)
        check(rsvResult.invoke(handle, out, maxSampleSize.toLong, n).asInstanceOf[Int])
        val len = n.get(JAVA_LONG, 0L)
        // Sampler.scala:330 wraps the samples array the same way (ArraySeq.ofLong / ofInt / ofRef)
        if (isUuid) {
          val w = out.asSlice(0L, len * 16).toArray(JAVA_LONG)
          ArraySeq.unsafeWrapArray(Array.tabulate(len.toInt)(i => new java.util.UUID(w(2 * i), w(2 * i + 1))))
        } else if (isLong) ArraySeq.unsafeWrapArray(out.asSlice(0L, len * 8).toArray(JAVA_LONG))
        else ArraySeq.unsafeWrapArray(out.asSlice(0L, len * 4).toArray(JAVA_INT))
      } finally tmp.close()
    if (!reusable) { // SingleUse.close: destroy now; `open` keeps every later call off the handle
      open = false
      cleanable.clean()
    }
    res.asInstanceOf[IndexedSeq[B]]
  }

  def isOpen: Boolean = open
}

/** Instantiated by gpu.Backend with Class.forName(...).getDeclaredConstructor().newInstance(): a class
  * with a no-argument constructor (private[reservoir] is public in bytecode).  Only this module
  * resolves java.lang.foreign. */
private[reservoir] final class FfmFactory extends SamplerFactory {
  def make[A, B](kind: Int, k: Int, reusable: Boolean, keys: KeyKind[B], hashKind: Int, engine: Int, seed: Long)(
      map: A => B,
      hash: B => Long,
  ): Sampler[A, B] = new FfmSampler[A, B](kind, k, reusable, keys, hashKind, engine, seed)(map, hash)

  def makeObjects[A, B: ClassTag](k: Int, reusable: Boolean, engine: Int, seed: Long)(map: A => B): Sampler[A, B] =
    new ObjectSampler[A, B](k, reusable, new FfmIndexOps(k, reusable, engine, seed))(map)
}

/** [[IndexOps]] over the FFM downcalls: an ELEMENTS handle (8-byte key width, never used for keys)
  * whose slots the engine fills by index only (rsv_commit_indexed); the B values live in the
  * [[ObjectSampler]].  The offsets come back through one native k-entry buffer. */
private[reservoir] final class FfmIndexOps(k: Int, reusable: Boolean, engine: Int, seed: Long) extends IndexOps {
  import Native._

  private[this] val arena = Arena.ofShared()
  private[this] val handle: MemorySegment = {
    val cfg = arena.allocate(Config)
    check(rsvConfigInit.invoke(cfg).asInstanceOf[Int])
    cfg.set(JAVA_INT, 4L, Abi.KindElements)
    cfg.set(JAVA_INT, 8L, k)
    cfg.set(JAVA_INT, 16L, if (reusable) 1 else 0)
    cfg.set(JAVA_INT, 24L, engine)
    cfg.set(JAVA_LONG, 40L, seed)
    val out = arena.allocate(ADDRESS)
    check(rsvCreate.invoke(cfg, out).asInstanceOf[Int])
    out.get(ADDRESS, 0L)
  }
  private[this] val offs = arena.allocate(8L * k, 8L)
  private[this] val cleanable = {
    val h = handle
    val a = arena
    cleaner.register(this, () => { rsvDestroy.invoke(h); a.close() })
  }

  def sampleIndexed(n: Long, offsets: Array[Long]): Unit = {
    check(rsvSampleIndexed.invoke(handle, n, offs).asInstanceOf[Int])
    MemorySegment.copy(offs, JAVA_LONG, 0L, offsets, 0, k)
  }
  def commitIndexed(): Unit = check(rsvCommitIndexed.invoke(handle).asInstanceOf[Int])
  def abortIndexed(): Unit  = check(rsvAbortIndexed.invoke(handle).asInstanceOf[Int])
  def release(): Unit       = cleanable.clean()
}
