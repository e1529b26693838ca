cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for e in 256 512; do for b in 0 1; do
  FAMG_DIA_BANDS=$b timeout -k 10 300 python bench.py --edge $e --steps 20 --warmup 3 --no-cpu-baseline --no-general > gpurun_out/ab_${e}_${b}.log 2>&1 || exit 1
  python - "$e" "$b" <<'PY'
import json,sys
l=[x for x in open(f"gpurun_out/ab_{sys.argv[1]}_{sys.argv[2]}.log") if x.startswith("{")][0]
d=json.loads(l); r=d["roofline"]
print(sys.argv[1], "bands", sys.argv[2], "cycle_ms", d["ms_per_step"], "fine_spmv_us", round(r["ms_per_launch"]*1e3,1), "frac", r["frac"])
PY
done; done
