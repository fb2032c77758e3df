"""Run bench.py with one engine class attribute changed, for in-call A/B
(profiling only): python profiles/bench_variant.py ATTR=VALUE -- <bench args>
e.g. overlap_store=0.  The package is loaded first and the attribute set on
TMREngine; bench.py then runs as __main__ in the same process."""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tmr_import import load_package  # noqa: E402

tmr = load_package()
i = sys.argv.index("--")
for kv in sys.argv[1:i]:
    k, v = kv.split("=", 1)
    setattr(tmr.TMREngine, k, type(getattr(tmr.TMREngine, k))(int(v)) if v.isdigit() else v)
sys.argv = [os.path.join(REPO, "bench.py")] + sys.argv[i + 1:]
runpy.run_path(sys.argv[0], run_name="__main__")
