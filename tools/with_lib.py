"""Run a script against another build of the engine (same-box A/B of dev variants):
    python tools/with_lib.py reservoir_amd/libreservoir_hip_exp.so tools/bench_paths.py --only c4o
The variant is built by `make -C reservoir_amd/csrc exp EXP="-D..."`; nothing in the product reads it."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    lib = os.path.abspath(sys.argv[1])
    from reservoir_amd import _native

    _native.LIB_PATH = lib
    sys.argv = sys.argv[2:]
    runpy.run_path(sys.argv[0], run_name="__main__")
