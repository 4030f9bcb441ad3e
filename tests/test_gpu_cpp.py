"""The C++ host mirror (include/reservoir/Sampler.hpp) compiled with g++ against the C ABI and run
on the GPU: reference boundary/lifecycle cases and oracle-checked reservoirs."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_compiles_without_gpu(tmp_path):
    exe = tmp_path / "t"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "cpp", "test_sampler.cpp"), "-o", str(exe),
                        "-L", os.path.join(ROOT, "reservoir_amd"), "-lreservoir_hip",
                        f"-Wl,-rpath,{os.path.join(ROOT, 'reservoir_amd')}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_cpp_mirror_on_gpu(tmp_path, cuda, oracle):
    exe = tmp_path / "t"
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "test_sampler.cpp"), "-o", str(exe),
                    "-L", os.path.join(ROOT, "reservoir_amd"), "-lreservoir_hip",
                    f"-Wl,-rpath,{os.path.join(ROOT, 'reservoir_amd')}"], check=True)
    lines = []
    for k, seed, stream, n in [(5, 1, 2, 1000), (1024, 0xC0FFEE, 0x5A5A, 200_000), (100, 7, 0, 99)]:
        keys = np.arange(n, dtype=np.int64)
        want, _ = oracle.algo_r(seed, stream, k, keys)
        lines.append(f"{k} {seed} {stream} {n}\n" + " ".join(str(int(v)) for v in want[: min(n, k)]))
    f = tmp_path / "cases.txt"
    f.write_text("\n".join(lines) + "\n")
    r = subprocess.run([str(exe), str(f)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
