"""Host replay forms of the ordered-distinct replica (rsv_host_values.h, Sampler.scala:394-409):
the set-based run and the heap-only run over first-occurrence flags leave identical heaps on
segments with repeated keys, members repeating across segments and tied hashes
(tests/cpp/test_host_replay.cpp, compiled here with g++; CPU only)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_replay_forms_identical(tmp_path):
    exe = tmp_path / "test_host_replay"
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-I", os.path.join(ROOT, "reservoir_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "test_host_replay.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok ")


def test_replay_forms_identical_sanitized(tmp_path):
    """The same host replica code under AddressSanitizer + UndefinedBehaviorSanitizer (host code only;
    the GPU side has no sanitizer on this pool): heap, slot pool and open-addressing table accesses
    stay in bounds and free of UB on tied, repeating segments and byte-row keys."""
    exe = tmp_path / "test_host_replay_asan"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                    "-fno-omit-frame-pointer", "-Wall", "-I", os.path.join(ROOT, "reservoir_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "test_host_replay.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok ")
