R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 120 python -u tools/pp_check.py 2>&1 | grep -v amdgpu.ids || exit 1
for i in 1 2; do for v in 0 1; do echo "== PP=$v"; LTX_ATTN_PP=$v timeout -k 10 120 python -u tools/attn_bench.py --which self --iters 30 2>&1 | grep -v amdgpu.ids || exit 1; done; done
