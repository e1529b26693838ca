#!/bin/bash
# round-6 GPU steps, each under its own time limit; stops after a step that
# faults, aborts or times out (exit codes other than 0 / 1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "== $name" >&2
    local t0=$(date +%s)
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    local t1=$(date +%s)
    echo "$name rc=$rc wall=$((t1 - t0))s" | tee -a gpurun_out/r6_steps_wall.txt
    tail -4 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
for s in "$@"; do
    case $s in
        fusetests) step r6_pytest_fuse 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 \
                   --timeout-method thread -k "fine_fused or cycle_plan_accounts or constant_diagonal or dia7_row or storage_mix or setdf or gtc or coarse_cholesky or spmm" ;;
        gputests) step r6_pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
        gputestsall) step r6_pytest_gpu 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
        tailtests) step r6_pytest_tail 600 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "dense_tail or cycle_plan or wide_grid or fold_zero" ;;
        profc2) step r6_profc2 400 bash scripts/prof_c2.sh r6_c2f ;;
        profc3) step r6_profc3 500 bash scripts/prof_c3.sh r6_c3f ;;
        profc5) step r6_profc5 500 bash scripts/prof_c5.sh r6_c5f ;;
        bench) step r6_bench 600 python bench.py --steps 20 --warmup 5 ;;
        pmc) step r6_pmc 600 bash scripts/pmc_cycle.sh ;;
        loop8) step r6_loop8 900 python bench.py --loopback 8 --steps 5 --warmup 1 ;;
        one512) step r6_one512 600 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline ;;
        spmm) step r6_spmm 300 python scripts/time_spmm.py ;;
        pmcfused) step r6_pmcfused 600 bash scripts/pmc_fused.sh ;;
        timefused) step r6_timefused 300 python scripts/time_fused.py 0 1 2 3 ;;
        timefused0) step r6_timefused 300 python scripts/time_fused.py 0 ;;
        pmcsq) step r6_pmcsq 400 bash scripts/pmc_cycle_sq.sh ;;
        abrows) step r6_abrows 400 bash scripts/r06_ab_rows.sh ;;
        smoke) step r6_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    esac
done
