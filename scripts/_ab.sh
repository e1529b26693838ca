set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "sgs" > gpurun_out/t_sgs.log 2>&1 || { tail -30 gpurun_out/t_sgs.log; exit 1; }
tail -n 1 gpurun_out/t_sgs.log
bash scripts/prof_c3.sh c3ex > /dev/null; grep -E "sgs27|per V-cycle" gpurun_out/c3ex.txt | head -2
grep '^{' gpurun_out/c3ex.log | cut -c1-160
