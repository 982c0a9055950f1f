"""One line per bench.py JSON file: value, ms/step and the kernels' ms/view (for sweeps)."""
import json
import sys

for path in sys.argv[1:]:
    lines = [ln for ln in open(path).read().splitlines() if ln.startswith("{")]
    if not lines:
        print(path, "no result")
        continue
    d = json.loads(lines[-1])
    kern = {k: v["ms_per_view"] for k, v in d.get("kernels", {}).items()}
    print(path, d["value"], d["ms_per_step"], kern)
