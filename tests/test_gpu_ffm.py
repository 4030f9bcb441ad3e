"""The JVM bindings' call sequences on the GPU (no JDK in the image): tests/cpp/test_ffm_sequence.cpp
replays the Panama FFM binding (FfmSampler.scala) and the JNI shim's session logic
(bindings/jvm/rsv_jvm.c, what every native method of bindings/jni/reservoir_jni.c calls) against
expected results the oracle computes here: element samplers (philox_r and the reference's
Algorithm L), distinct samplers with each hash kind (default Long/Int hashCode, identity,
precomputed), single-use lifecycle (isOpen false, IllegalStateException after result(), the handle
never touched after it is destroyed) and reusable results; plus C5's k = 1 Mi through per-element
rsv_sample and through FFM staging."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HASH_DEFAULT, HASH_IDENTITY, HASH_JAVA_LONG, HASH_JAVA_INT, HASH_PRECOMPUTED = range(5)


def build(tmp_path):
    obj = tmp_path / "rsv_jvm.o"
    exe = tmp_path / "ffm"
    r = subprocess.run(["gcc", "-std=c11", "-O2", "-Wall", "-c", os.path.join(ROOT, "bindings", "jvm", "rsv_jvm.c"),
                        "-o", str(obj)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", os.path.join(ROOT, "tests", "cpp", "test_ffm_sequence.cpp"),
                        str(obj), "-o", str(exe), "-L", os.path.join(ROOT, "reservoir_amd"), "-lreservoir_hip",
                        f"-Wl,-rpath,{os.path.join(ROOT, 'reservoir_amd')}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_bindings_compile_without_gpu(tmp_path):
    """The JNI session glue and the call-sequence harness build against the C ABI here (CPU)."""
    build(tmp_path)


def _keys(oracle, base, n, kw):
    k = oracle.splitmix_keys(base, n)
    return k if kw == 8 else (k >> 33).astype(np.int32)


@pytest.mark.gpu
def test_ffm_and_jni_call_sequences(tmp_path, cuda, oracle):
    exe = build(tmp_path)
    cases = []

    def add(name, path, kind, k, kw, reusable, hash_kind, engine, seed, stream, n, base, want):
        f = tmp_path / f"{name}.bin"
        np.ascontiguousarray(want, dtype=np.int64 if kw == 8 else np.int32).tofile(f)
        cases.append(f"{name} {path} {kind} {k} {kw} {reusable} {hash_kind} 0 {engine} {seed} {stream} {n} {base} {f}")

    def elements(seed, stream, k, keys):
        win = oracle.algo_r_last_writers(seed, stream, k, 0, keys.size)
        return keys[win[win >= 0]]

    # element samplers (Sampler.apply)
    x = _keys(oracle, 0x5EED0000, 3_000_000, 8)
    want = elements(0xC0FFEE, 0x5A5A, 1024, x)
    add("ffm_elements_long", "ffm", 0, 1024, 8, 0, 0, 0, 0xC0FFEE, 0x5A5A, x.size, 0x5EED0000, want)
    add("jni_elements_long", "jni", 0, 1024, 8, 0, 0, 0, 0xC0FFEE, 0x5A5A, x.size, 0x5EED0000, want)
    x = _keys(oracle, 77, 2_000_003, 4)
    want = elements(5, 6, 777, x)
    add("ffm_elements_int_reusable", "ffm", 0, 777, 4, 1, 0, 0, 5, 6, x.size, 77, want)
    add("jni_elements_int_reusable", "jni", 0, 777, 4, 1, 0, 0, 5, 6, x.size, 77, want)
    x = _keys(oracle, 9, 1_000_000, 8)
    ref = oracle.AlgoL(100, 0)
    ref.sample_all(x)
    add("ffm_elements_java_l", "ffm", 0, 100, 8, 0, 0, 1, 0, 0, x.size, 9, ref.result())
    add("jni_elements_java_l", "jni", 0, 100, 8, 0, 0, 1, 0, 0, x.size, 9, ref.result())
    # C5: k = 1 Mi over 3e7 keys, per-element rsv_sample and FFM staging
    x = _keys(oracle, 0xC5, 30_000_000, 8)
    want = elements(21, 3, 1 << 20, x)
    add("abi_c5_k1mi", "abi", 0, 1 << 20, 8, 0, 0, 0, 21, 3, x.size, 0xC5, want)
    add("ffm_c5_k1mi", "ffm", 0, 1 << 20, 8, 0, 0, 0, 21, 3, x.size, 0xC5, want)

    # distinct samplers (Sampler.distinct), every hash kind the bindings pass through
    def distinct(kw, hash_kind, seed, k, n, base, path):
        xs = _keys(oracle, base, n, kw)
        xs = np.concatenate([xs, xs[: n // 3]])  # duplicates
        if hash_kind == HASH_PRECOMPUTED:  # hash = 31 x + 7 (a bijection of Long)
            ys = xs.astype(np.int64) * 31 + 7
            ref = oracle.Distinct(k, seed, oracle.HASH_IDENTITY)
            ref.sample_all(ys)
            back = dict(zip(ys.tolist(), xs.tolist()))
            want = np.sort([back[y] for y in ref.result()[0].tolist()])
        else:
            ok = {HASH_DEFAULT: oracle.HASH_JAVA_LONG if kw == 8 else oracle.HASH_JAVA_INT,
                  HASH_IDENTITY: oracle.HASH_IDENTITY, HASH_JAVA_INT: oracle.HASH_JAVA_INT}[hash_kind]
            ref = oracle.Distinct(k, seed, ok)
            ref.sample_all(xs.astype(np.int64))
            want = np.sort(ref.result()[0])
        name = f"{path}_distinct_kw{kw}_hash{hash_kind}"
        f = tmp_path / f"{name}.bin"
        want.astype(np.int64 if kw == 8 else np.int32).tofile(f)
        # the harness regenerates keys 0..n-1, then the duplicates: write them out instead
        kf = tmp_path / f"{name}.keys"
        xs.tofile(kf)
        cases.append(f"{name} {path} 1 {k} {kw} 0 {hash_kind} 0 0 {seed} 0 {xs.size} 0 {f} {kf}")

    # java.util.UUID keys (KeyKind.UuidKey, 16 bytes [msb | lsb]): the harness writes key i as
    # [v_i, ~v_i], v_i = splitmix64(base + i); the default hash is UUID.hashCode (on the GPU), a
    # precomputed one 31 v + 7
    def uuid_distinct(hash_kind, seed, k, n, base, path):
        v = oracle.splitmix_keys(base, n)
        v = np.concatenate([v, v[: n // 3]])
        rows = np.stack([v, ~v], axis=1)
        if hash_kind == HASH_DEFAULT:
            ref = oracle.DistinctRows(k, seed, 16, "uuid")
            ref.sample_all(rows.view(np.uint8))
        else:
            ref = oracle.DistinctRows(k, seed, 16)
            ref.sample_all(rows.view(np.uint8), v * 31 + 7)
        name = f"{path}_distinct_uuid_hash{hash_kind}"
        f = tmp_path / f"{name}.bin"
        ref.result()[0].tofile(f)
        kf = tmp_path / f"{name}.keys"
        rows.tofile(kf)
        cases.append(f"{name} {path} 1 {k} 16 0 {hash_kind} 0 0 {seed} 0 {v.size} 0 {f} {kf}")

    for path in ("ffm", "jni"):
        uuid_distinct(HASH_DEFAULT, 8, 3000, 400_000, 35, path)
        uuid_distinct(HASH_PRECOMPUTED, 9, 1000, 300_000, 36, path)
    # UUID element samplers: key i = [v_i, ~v_i]
    for path in ("ffm", "jni"):
        v = oracle.splitmix_keys(37, 1_000_000)
        win = oracle.algo_r_last_writers(11, 12, 500, 0, v.size)
        want = np.stack([v[win], ~v[win]], axis=1)
        f = tmp_path / f"{path}_elements_uuid.bin"
        want.tofile(f)
        cases.append(f"{path}_elements_uuid {path} 0 500 16 0 0 0 0 11 12 {v.size} 37 {f}")
    for path in ("ffm", "jni"):
        distinct(8, HASH_DEFAULT, 3, 5000, 600_000, 31, path)
        distinct(8, HASH_IDENTITY, 4, 4096, 500_000, 32, path)
        distinct(4, HASH_DEFAULT, 5, 3000, 400_000, 33, path)
        distinct(8, HASH_PRECOMPUTED, 6, 2000, 300_000, 34, path)
    f = tmp_path / "cases.txt"
    f.write_text("\n".join(cases) + "\n")
    r = subprocess.run([str(exe), str(f)], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("PASS") == len(cases), r.stdout


@pytest.mark.gpu
def test_indexed_sample_all_through_the_bindings(tmp_path, cuda, oracle):
    """sampleAll over an IndexedSeq through both JVM paths (FfmSampler.sampleAll's downcalls and
    JniSampler's natives over rsv_jvm): rsv_sample_indexed + rsv_fill_slots, the sequence virtual
    (no key buffer: the harness computes key i only when the engine names offset i).  At C2's shape
    -- a 1e9-element sequence, k = 1024 -- the reservoir must equal the oracle's last writers
    (philox_r) and the oracle's own sampleIndexed walk of Algorithm L (java_l, Sampler.scala:261-273),
    with map run for at most k elements.  Small cases cover n < k, n = k and Int keys."""
    exe = build(tmp_path)
    sm = oracle.lib().or_splitmix64
    cases = []

    def key_of(base, i, kw):
        v = np.array([sm(base + int(i))], dtype=np.uint64).view(np.int64)[0]
        return int(v) if kw == 8 else int(v) >> 33

    def add(name, path, k, kw, engine, seed, stream, n, base, idx):
        want = np.array([key_of(base, i, kw) for i in idx.tolist()], dtype=np.int64 if kw == 8 else np.int32)
        f = tmp_path / f"{name}.bin"
        want.tofile(f)
        cases.append(f"{name} {path} 0 {k} {kw} 0 0 0 {engine} {seed} {stream} {n} {base} {f}")

    n = 1_000_000_000
    win = oracle.algo_r_last_writers(0xC0FFEE, 0x5A5A, 1024, 0, n)
    assert (win >= 0).all()
    ref = oracle.AlgoL(1000, 0)
    ref.sample_all_iota(0, n)
    for path in ("fidx", "jidx"):
        add(f"{path}_c2_philox", path, 1024, 8, 0, 0xC0FFEE, 0x5A5A, n, 0x5EED0000, win)
        add(f"{path}_c2_java_l", path, 1000, 8, 1, 0, 0, n, 0x5EED0000, ref.result())
    for n_small, k in ((500, 1024), (1024, 1024), (70_001, 64)):
        w = oracle.algo_r_last_writers(7, 8, k, 0, n_small)
        add(f"jidx_small_{n_small}_{k}", "jidx", k, 4, 0, 7, 8, n_small, 99, w[w >= 0])
        r = oracle.AlgoL(k, 3)
        r.sample_all_iota(0, n_small)
        add(f"fidx_small_java_l_{n_small}_{k}", "fidx", k, 8, 1, 3, 0, n_small, 5, r.result())
    f = tmp_path / "cases.txt"
    f.write_text("\n".join(cases) + "\n")
    r = subprocess.run([str(exe), str(f)], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("PASS") == len(cases), r.stdout


@pytest.mark.gpu
def test_object_sampler_call_sequences(tmp_path, cuda, oracle):
    """A Sampler[A, B] for any B (ObjectSampler.scala, round 6): the engine decides which element
    each slot holds from the indices alone (rsv_sample_indexed + rsv_commit_indexed) and the JVM
    keeps the B values.  With element i standing for the reference i, the reservoir must be the
    oracle's last-writer indices (philox_r) and the reference's own Algorithm-L sampleIndexed walk
    (java_l, Sampler.scala:261-273) -- at C2's 1e9 elements on both JVM paths, after buffered
    sample() batches and a first sampleAll whose map throws (rsv_abort_indexed undoes it)."""
    exe = build(tmp_path)
    cases = []

    def add(name, path, k, reusable, engine, seed, stream, n, want):
        f = tmp_path / f"{name}.bin"
        np.ascontiguousarray(want, dtype=np.int64).tofile(f)
        cases.append(f"{name} {path} 0 {k} 8 {reusable} 0 0 {engine} {seed} {stream} {n} 0 {f}")

    n = 1_000_000_000
    win = oracle.algo_r_last_writers(0xC0FFEE, 0x5A5A, 1024, 0, n)
    ref = oracle.AlgoL(1000, 0)
    ref.sample_all_iota(0, n)
    for path in ("fobj", "jobj"):
        add(f"{path}_c2_philox", path, 1024, 0, 0, 0xC0FFEE, 0x5A5A, n, win)
        add(f"{path}_c2_java_l", path, 1000, 1, 1, 0, 0, n, ref.result())
    for n_small, k in ((500, 1024), (100_003, 70_000), (300_000, 64), (2_000_000, 100_000)):
        w = oracle.algo_r_last_writers(7, 8, k, 0, n_small)
        add(f"fobj_small_{n_small}_{k}", "fobj", k, 1, 0, 7, 8, n_small, w[w >= 0])
        r = oracle.AlgoL(k, 3)
        r.sample_all_iota(0, n_small)
        add(f"jobj_small_java_l_{n_small}_{k}", "jobj", k, 0, 1, 3, 0, n_small, r.result())
    f = tmp_path / "cases.txt"
    f.write_text("\n".join(cases) + "\n")
    r = subprocess.run([str(exe), str(f)], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("PASS") == len(cases), r.stdout
