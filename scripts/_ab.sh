set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "dia27 or 27pt or sgs27 or dia_codes or dia" > gpurun_out/t_cst.log 2>&1 || { tail -30 gpurun_out/t_cst.log; exit 1; }
tail -n 1 gpurun_out/t_cst.log
bash scripts/prof_c3.sh c3cst > /dev/null; grep -E "dia_pat|per V-cycle" gpurun_out/c3cst.txt | head -3
FAMG_DIA_CST=0 bash scripts/prof_c3.sh c3nocst > /dev/null; grep -E "dia_pat|per V-cycle" gpurun_out/c3nocst.txt | head -3
