set -e
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu.log
bash scripts/prof_c2.sh c2sd > /dev/null; grep -E "per V-cycle|SETDF|k_mul2" gpurun_out/c2sd.txt | head -8
bash scripts/prof_c3.sh c3sd > /dev/null; grep -E "per V-cycle|SETDF|k_mul2" gpurun_out/c3sd.txt | head -8
