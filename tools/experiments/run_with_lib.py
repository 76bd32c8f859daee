"""Run a script (bench.py, bench_configs.py, or -m pytest ...) against another build of the library, e.g. an
ablation from fir_ablate.sh: python tools/experiments/run_with_lib.py LIB.so SCRIPT [args].
The package loads its library at import, so sdrgpu._lib is pre-seeded in sys.modules with
LIB_PATH pointing at LIB.so before the package itself is imported."""
import importlib.util
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "unnamed-rust-sdr_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)
spec = importlib.util.spec_from_file_location("sdrgpu._lib", os.path.join(PKG, "sdrgpu", "_lib.py"))
mod = importlib.util.module_from_spec(spec)
sys.modules["sdrgpu._lib"] = mod
spec.loader.exec_module(mod)
mod.LIB_PATH = os.path.abspath(sys.argv[1])
import sdrgpu  # noqa: E402,F401  (package init now loads LIB.so)
assert sdrgpu._lib.lib()._name == mod.LIB_PATH, "variant library not loaded"
print(f"[run_with_lib] {mod.LIB_PATH}", file=sys.stderr)
sys.argv = sys.argv[2:]
if sys.argv[0] == "-m":  # a module, e.g. -m pytest ...
    sys.argv = sys.argv[1:]
    runpy.run_module(sys.argv[0], run_name="__main__", alter_sys=True)
else:
    runpy.run_path(sys.argv[0], run_name="__main__")
