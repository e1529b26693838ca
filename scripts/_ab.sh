set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -k "gtc or grid_transfer or setdf or transfer or constant_diagonal or slab or one_rank or vcycle_256" > gpurun_out/t_gtc.log 2>&1 || { tail -30 gpurun_out/t_gtc.log; exit 1; }
tail -n 1 gpurun_out/t_gtc.log
bash scripts/prof_c2.sh c2rm > /dev/null; grep -E "restrict_march|per V-cycle" gpurun_out/c2rm.txt | head -2
bash scripts/prof_c3.sh c3rm > /dev/null; grep -E "restrict_march|per V-cycle" gpurun_out/c3rm.txt | head -2
FAMG_GTC_NT=1 bash scripts/prof_c2.sh c2nt > /dev/null; grep -E "gtc_interp|per V-cycle" gpurun_out/c2nt.txt | head -3
