set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -k "gtc or grid_transfer or setdf or transfer or constant_diagonal or slab or one_rank or vcycle_256" > gpurun_out/t_gtc.log 2>&1 || { tail -30 gpurun_out/t_gtc.log; exit 1; }
tail -n 1 gpurun_out/t_gtc.log
bash scripts/prof_c2.sh c2xp2 > /dev/null; grep -E "gtc_interp|per V-cycle" gpurun_out/c2xp2.txt | head -3
FAMG_GTC_XP=1 bash scripts/prof_c2.sh c2xp1 > /dev/null; grep -E "gtc_interp|per V-cycle" gpurun_out/c2xp1.txt | head -3
bash scripts/prof_c3.sh c3xp2 > /dev/null; grep -E "gtc_interp|per V-cycle" gpurun_out/c3xp2.txt | head -3
