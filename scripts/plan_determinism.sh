#!/bin/bash
# Two plain bench runs and one under counter collection (rocprofv3 --pmc):
# their launch plans and per-level storages must agree (verdict r04 item 6)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
B="--steps 5 --warmup 2 --no-cpu-baseline --no-general --no-abi"
timeout -k 10 300 python3 bench.py $B > gpurun_out/pd_a.json 2> gpurun_out/pd_a.err || exit 1
timeout -k 10 300 python3 bench.py $B > gpurun_out/pd_b.json 2> gpurun_out/pd_b.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pd_pmc" -o run --output-format csv \
    -- python3 "$R/bench.py" $B > gpurun_out/pd_c.json 2> gpurun_out/pd_c.err || exit 1
python3 - <<'PY'
import json
runs = {k: json.load(open(f"gpurun_out/pd_{k}.json")) for k in "abc"}
plan = {k: v["config"]["vcycle_plan"] for k, v in runs.items()}
same_k = plan["a"]["per_level_kernels"] == plan["b"]["per_level_kernels"] == plan["c"]["per_level_kernels"]
same_s = plan["a"]["per_level_storage"] == plan["b"]["per_level_storage"] == plan["c"]["per_level_storage"]
out = {"runs": {"a": "bench.py", "b": "bench.py again (new process)", "c": "bench.py under rocprofv3 --pmc FETCH_SIZE"},
       "same_per_level_kernels": same_k, "same_per_level_storage": same_s,
       "per_level_kernels": plan["a"]["per_level_kernels"], "per_level_storage": plan["a"]["per_level_storage"],
       "vcycles_per_s": {k: v["value"] for k, v in runs.items()}}
json.dump(out, open("gpurun_out/plan_determinism.json", "w"), indent=1)
print(json.dumps({k: out[k] for k in ("same_per_level_kernels", "same_per_level_storage", "vcycles_per_s")}))
PY
