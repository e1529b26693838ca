cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -q --timeout 200 --timeout-method thread -k "stencil or class or scs or vcycle_256 or spmm or sgs27 or dist_stencil" > gpurun_out/t_scs.log 2>&1
echo "pytest rc=$?"
bash scripts/ab_sgs27.sh
bash scripts/gpu_check.sh profp
