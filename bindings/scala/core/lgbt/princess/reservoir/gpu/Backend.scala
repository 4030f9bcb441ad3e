package lgbt.princess.reservoir.gpu

import java.security.SecureRandom

import scala.reflect.ClassTag

import lgbt.princess.reservoir.Sampler

/** What a binding provides: a GPU sampler for one factory call.  The JNI binding lives in `core`
  * (JDK 8+); the Panama FFM one (JDK 22+, `java.lang.foreign`) is a separate sbt module
  * (`reservoir-gpu-ffm`, INTEGRATION.md) that `Backend` loads by name, so `core` itself never
  * references `java.lang.foreign` and still compiles on the reference's CI JDKs 8/11/15 under
  * `-Xlint -Werror` (build.sbt:37-42, :129-133). */
private[reservoir] trait SamplerFactory {
  def make[A, B](kind: Int, k: Int, reusable: Boolean, keys: KeyKind[B], hashKind: Int, engine: Int, seed: Long)(
      map: A => B,
      hash: B => Long,
  ): Sampler[A, B]

  /** Sampler.apply for a `B` with no fixed-width key: index-only batches, the elements kept on the
    * JVM ([[ObjectSampler]]) */
  def makeObjects[A, B: ClassTag](k: Int, reusable: Boolean, engine: Int, seed: Long)(map: A => B): Sampler[A, B]
}

private[reservoir] object JniFactory extends SamplerFactory {
  def make[A, B](kind: Int, k: Int, reusable: Boolean, keys: KeyKind[B], hashKind: Int, engine: Int, seed: Long)(
      map: A => B,
      hash: B => Long,
  ): Sampler[A, B] = new JniSampler[A, B](kind, k, reusable, keys, hashKind, engine, seed)(map, hash)

  def makeObjects[A, B: ClassTag](k: Int, reusable: Boolean, engine: Int, seed: Long)(map: A => B): Sampler[A, B] =
    new ObjectSampler[A, B](k, reusable, new JniIndexOps(k, reusable, engine, seed))(map)
}

/** Backend selection behind the unchanged factories `Sampler.apply` / `Sampler.distinct`
  * (Sampler.scala:128-136, :171-180; SURVEY.md section 5 "Config / flags"): no signature changes.
  *
  *   -Dreservoir.backend=gpu        use the MI355X engine: Sampler.apply for every B (Long, Int and
  *                                  java.util.UUID keys live on the GPU; any other B is sampled by
  *                                  index and its elements stay on the JVM, ObjectSampler);
  *                                  Sampler.distinct for B = Long, Int or UUID (else the JVM classes)
  *   -Dreservoir.binding=ffm|jni    default: FFM when the JDK is 22+ and the reservoir-gpu-ffm jar is
  *                                  on the class path, JNI otherwise
  *   -Dreservoir.engine=java_l      the reference's Algorithm L over java.util.Random, bit-identical
  *                                  to the JVM sampler for the same seed (default philox_r: Algorithm R)
  *
  * The akka operators need nothing: they take the sampler by name (Sample.scala:23-24,
  * SampleImpl.scala:10), so `Sample(k)(map)` picks the backend through `Sampler.apply`. */
private[reservoir] object Backend {
  private[this] val enabled = System.getProperty("reservoir.backend", "cpu") == "gpu"
  private[this] val FfmFactoryClass = "lgbt.princess.reservoir.gpu.ffm.FfmFactory"

  /** The FFM factory, loaded reflectively: absent module or pre-22 JDK -> JNI. */
  private[this] lazy val factory: SamplerFactory = {
    val wantFfm = System.getProperty("reservoir.binding") match {
      case "ffm" => true
      case "jni" => false
      case _ =>
        val v = System.getProperty("java.specification.version", "1.8")
        !v.startsWith("1.") && v.toInt >= 22
    }
    if (!wantFfm) JniFactory
    else
      try Class.forName(FfmFactoryClass).getDeclaredConstructor().newInstance().asInstanceOf[SamplerFactory]
      catch {
        case _: ReflectiveOperationException | _: LinkageError =>
          if (System.getProperty("reservoir.binding") == "ffm")
            throw new UnsupportedOperationException(
              s"-Dreservoir.binding=ffm needs JDK 22+ and $FfmFactoryClass (reservoir-gpu-ffm) on the class path"
            )
          JniFactory
      }
  }
  private[this] val engine = if (System.getProperty("reservoir.engine", "") == "java_l") Abi.EngineJavaL else Abi.EnginePhiloxR
  private[this] val seeds  = new SecureRandom() // a fresh seed per sampler, like `new Random()` (Sampler.scala:199)

  private[this] def make[A, B](kind: Int, k: Int, reusable: Boolean, keys: KeyKind[B], hashKind: Int)(
      map: A => B,
      hash: B => Long,
  ): Sampler[A, B] = {
    val seed = seeds.nextLong()
    factory.make[A, B](kind, k, reusable, keys, hashKind, engine, seed)(map, hash)
  }

  /** Sampler.apply (validation already done by validateNonDistinctParams). */
  def elements[A, B: ClassTag](maxSampleSize: Int, reusable: Boolean)(map: A => B): Option[Sampler[A, B]] =
    if (!enabled) None
    else
      KeyKind.of[B] match {
        case Some(kk) => Some(make[A, B](Abi.KindElements, maxSampleSize, reusable, kk, Abi.HashDefault)(map, null))
        case None => // any other B: which element each slot holds is decided on the GPU, the B stays here
          Some(factory.makeObjects[A, B](maxSampleSize, reusable, engine, seeds.nextLong())(map))
      }

  /** Sampler.distinct: the default `hashCode` and the identity hash run on the GPU; any other `hash`
    * is evaluated here per element and shipped beside the key (RSV_HASH_PRECOMPUTED). */
  def distinct[A, B: ClassTag](maxSampleSize: Int, reusable: Boolean)(map: A => B, hash: B => Long)(
      defaultHash: Any => Long
  ): Option[Sampler[A, B]] =
    if (!enabled) None
    else
      KeyKind.of[B].map { kk =>
        val hashKind =
          if (hash eq defaultHash) Abi.HashDefault
          else if (kk == KeyKind.LongKey && (hash eq Hashes.identity)) Abi.HashIdentity
          else Abi.HashPrecomputed
        make[A, B](Abi.KindDistinct, maxSampleSize, reusable, kk, hashKind)(map, hash)
      }
}
