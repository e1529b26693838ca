set -e
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu.log
bash scripts/prof_c2.sh c2cst > /dev/null; grep -E "dia_kernel|per V-cycle" gpurun_out/c2cst.txt | head -4
FAMG_DIA_CST=0 bash scripts/prof_c2.sh c2nocst > /dev/null; grep -E "dia_kernel|per V-cycle" gpurun_out/c2nocst.txt | head -4
