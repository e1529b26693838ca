set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "xstaged or stencil_classes" > gpurun_out/t_ug.log 2>&1 || { tail -30 gpurun_out/t_ug.log; exit 1; }
tail -n 1 gpurun_out/t_ug.log
bash scripts/prof_c3.sh c3ug16 > /dev/null; grep -E "xscs|per V-cycle" gpurun_out/c3ug16.txt | head -5
FAMG_LIB=$PWD/faer-amg_amd/build_ab/lib_ug8.so bash scripts/prof_c3.sh c3ug8 > /dev/null; grep -E "xscs|per V-cycle" gpurun_out/c3ug8.txt | head -5
bash scripts/prof_c2.sh c2ug16 > /dev/null; grep -E "xscs|per V-cycle" gpurun_out/c2ug16.txt | head -7
FAMG_LIB=$PWD/faer-amg_amd/build_ab/lib_ug8.so bash scripts/prof_c2.sh c2ug8 > /dev/null; grep -E "xscs|per V-cycle" gpurun_out/c2ug8.txt | head -7
