package lgbt.princess.reservoir.gpu

import scala.reflect.ClassTag

/** Constants of the C ABI (include/reservoir_hip.h) and the key kinds the engine stores.
  *
  * The engine keeps fixed-width keys only: `B = Long` (8 bytes), `B = Int` (4 bytes) or
  * `B = java.util.UUID` (16 bytes, [mostSigBits | leastSigBits]), which `map` extracts on the JVM
  * (Sampler.scala:115-116 allows `map` to run more than `maxSampleSize` times).
  */
private[reservoir] object Abi {
  // rsv_status -> the reference's exceptions (Sampler.scala:80-82, :94, :186)
  final val Ok               = 0
  final val IllegalArgument  = 1
  final val IllegalState     = 2
  final val NullPointer      = 3
  final val Device           = 4
  final val OutOfMemory      = 5
  final val Unsupported      = 6
  // rsv_kind
  final val KindElements = 0
  final val KindDistinct = 1
  // rsv_engine
  final val EnginePhiloxR = 0
  final val EngineJavaL   = 1
  // rsv_hash_kind
  final val HashDefault     = 0 // B#hashCode().toLong (Sampler.scala:75): Long / Int / UUID hashCode on the GPU
  final val HashIdentity    = 1
  final val HashJavaLong    = 2
  final val HashJavaInt     = 3
  final val HashPrecomputed = 4 // any other JVM `hash`: evaluated per element here, shipped beside the key
  // rsv_distinct_order
  final val OrderAuto = 0

  val ClosedMessage = "use of sampler after calling `result()`" // Sampler.scala:186

  def exception(status: Int, msg: String): Throwable = status match {
    case IllegalArgument => new IllegalArgumentException(msg)
    case IllegalState    => new IllegalStateException(msg)
    case NullPointer     => new NullPointerException(msg)
    case OutOfMemory     => new OutOfMemoryError(msg)
    case Unsupported     => new UnsupportedOperationException(msg)
    case _               => new RuntimeException(msg) // a device error fails the akka Future (SampleImpl.scala:43-46)
  }
}

/** How a stored element travels: its width and how it is written into / read out of native memory. */
private[reservoir] sealed abstract class KeyKind[B](val width: Int)

private[reservoir] object KeyKind {
  case object LongKey extends KeyKind[Long](8)
  case object IntKey  extends KeyKind[Int](4)

  /** java.util.UUID as two Longs, [mostSigBits | leastSigBits]: UUID.equals is equality of both
    * words, so the engine's byte equality is the reference's `elements.contains` (Sampler.scala:398,
    * :403), and its default hash is UUID.hashCode computed on the GPU.  (An Array[Byte] has
    * reference equality in a Scala Set: it never maps to a key kind and stays on the JVM classes.) */
  case object UuidKey extends KeyKind[java.util.UUID](16)

  def of[B](implicit ct: ClassTag[B]): Option[KeyKind[B]] =
    if (ct == ClassTag.Long) Some(LongKey.asInstanceOf[KeyKind[B]])
    else if (ct == ClassTag.Int) Some(IntKey.asInstanceOf[KeyKind[B]])
    else if (ct.runtimeClass == classOf[java.util.UUID]) Some(UuidKey.asInstanceOf[KeyKind[B]])
    else None
}

/** The identity hash for `Sampler.distinct(k)(map, gpu.Hashes.identity)`: recognised by reference
  * equality and computed on the GPU (a bijection of Long: bit-exact, order-independent sets). */
object Hashes {
  val identity: Long => Long = (x: Long) => x
}
