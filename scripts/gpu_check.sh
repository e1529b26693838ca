#!/bin/bash
# GPU-box check: each GPU step under its own time limit; stop at the first
# step that faults, aborts or times out (exit codes other than 0/1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "== $name" >&2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
for s in "$@"; do
    case $s in
        tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
        satests) step pytest_sa 600 python -u -m pytest tests/test_gpu_sa.py tests/test_gpu_dist.py -m gpu -v --timeout 120 --timeout-method thread ;;
        elast30) step bench_elast30 400 python bench.py --problem elast --elements 30 --steps 20 --warmup 3 ;;
        elast) step bench_elast 900 python bench.py --problem elast --steps 20 --warmup 3 ;;
        c4one) step bench_c4one 600 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline ;;
        dist1c4) step dist1c4 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
                  --master-addr 127.0.0.1 --master-port 29515 bench.py --dist --workload c4 --steps 5 --warmup 1 ;;
        benchg) step bench_g 500 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
        prof27) export TMPDIR=/tmp; R=$(pwd)
              step prof27 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof27" -o run \
                  --output-format csv -- python3 "$R/bench.py" --problem 27pt --smoother sgs --steps 10 --warmup 2 --no-cpu-baseline ;;
        profelast) export TMPDIR=/tmp; R=$(pwd)
              step profelast 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profelast" -o run \
                  --output-format csv -- python3 "$R/bench.py" --problem elast --steps 20 --warmup 3 --no-cpu-baseline ;;
        plantest) step plantest 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 \
                  --timeout-method thread -k "cycle_plan" ;;
        launch1) step launch1 600 python bench.py --gpus 1 --dist --steps 20 --warmup 3 ;;
        launch1c4) step launch1c4 600 python bench.py --gpus 1 --dist --workload c4 --steps 5 --warmup 1 ;;
        profp) export TMPDIR=/tmp; R=$(pwd)
              step profp 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profp" -o run \
                  --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-general \
                  --plan-out "$R/gpurun_out/plan_c2.json" ;;
        profp27) export TMPDIR=/tmp; R=$(pwd)
              step profp27 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profp27" -o run \
                  --output-format csv -- python3 "$R/bench.py" --problem 27pt --steps 10 --warmup 2 --no-cpu-baseline \
                  --no-general --plan-out "$R/gpurun_out/plan_c3.json" ;;
        profpel) export TMPDIR=/tmp; R=$(pwd)
              step profpel 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profpel" -o run \
                  --output-format csv -- python3 "$R/bench.py" --problem elast --steps 20 --warmup 3 --no-cpu-baseline \
                  --plan-out "$R/gpurun_out/plan_c5.json" ;;
        ptk) step ptk 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -k "$PTK" ;;
        absgs) step absgs 900 bash scripts/ab_sgs27.sh ;;
        bench27g) step bench27g 600 python bench.py --problem 27pt --smoother sgs --steps 10 --warmup 2 --no-cpu-baseline --no-general ;;
        pmcbsr) export TMPDIR=/tmp; R=$(pwd)
              step pmcbsr_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmcbsr_fetch" -o run \
                  --output-format csv -- python3 "$R/scripts/pmc_bsr.py"
              step pmcbsr_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmcbsr_write" -o run \
                  --output-format csv -- python3 "$R/scripts/pmc_bsr.py" ;;
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) step bench 600 python bench.py --steps 20 --warmup 3 ;;
        benchq) step bench 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --ab ;;
        dist2) step dist2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --edge 64 --steps 5 --warmup 1 ;;
        benchnolds) FAMG_DIA_LDS=0 step bench_nolds 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
        levelinfo) step levelinfo 300 python scripts/level_info.py ;;
        dist1) step dist1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
                  --master-addr 127.0.0.1 --master-port 29513 bench.py --dist --edge 256 --steps 10 --warmup 2 ;;
        ablevels) step ablevels 400 python scripts/ab_levels.py ;;
        pstream) step pstream 300 python scripts/placement_stream.py ;;
        placement) FAMG_ALLOC_DEBUG=1 step placement 300 python scripts/placement.py ;;
        bench27) step bench27 600 python bench.py --problem 27pt --smoother sgs --steps 10 --warmup 2 --no-cpu-baseline ;;
        bench27p) step bench27p 900 python bench.py --problem 27pt --smoother sgs --steps 10 --warmup 2 --cpu-budget 4 --no-general ;;
        bench512) step bench512 600 python bench.py --edge 512 --steps 5 --warmup 1 --no-cpu-baseline ;;
        benchblock) step benchblock 600 python bench.py --smoother block --steps 10 --warmup 2 --no-cpu-baseline ;;
        pmc) export TMPDIR=/tmp; R=$(pwd)
              step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmc_fetch" -o run \
                  --output-format csv -- python3 "$R/scripts/pmc_fine_spmv.py"
              step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmc_write" -o run \
                  --output-format csv -- python3 "$R/scripts/pmc_fine_spmv.py" ;;
        prof) export TMPDIR=/tmp; R=$(pwd)
              step prof 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run \
                  --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline ;;
    esac
done
