set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "gtc or grid_transfer or setdf or transfer or constant_diagonal" > gpurun_out/t_gtc.log 2>&1 || { tail -30 gpurun_out/t_gtc.log; exit 1; }
tail -n 1 gpurun_out/t_gtc.log
FAMG_GTC_E32=1 bash scripts/prof_c2.sh c2e1
FAMG_GTC_E32=0 bash scripts/prof_c2.sh c2e0
FAMG_GTC_E32=1 FAMG_GTC_RTZ=4 bash scripts/prof_c2.sh c2e1r4
