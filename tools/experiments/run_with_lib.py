"""Run a script (bench.py, bench_configs.py) against another build of the library, e.g. an
ablation from fir_ablate.sh: python tools/experiments/run_with_lib.py LIB.so SCRIPT [args]."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unnamed-rust-sdr_amd"))
sys.path.insert(0, ROOT)
import sdrgpu._lib as L  # noqa: E402

L.LIB_PATH = os.path.abspath(sys.argv[1])
sys.argv = sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
