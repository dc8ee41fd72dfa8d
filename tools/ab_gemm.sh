R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for v in 4 8; do echo "== lora rows sched $v"; LTX_LORA_ROWS=$v timeout -k 10 120 python -u tools/lora_bench.py || exit $?; done
for i in 1 2; do for L in build_exp/base.so build_exp/ilv/libltxhip.so; do
  echo "== gemm $L"; LTX_HIP_LIB=$L timeout -k 10 120 python -u tools/bench_gemm.py | grep -v "^{" || exit $?
done; done
for i in 1 2; do for L in build_exp/base.so build_exp/ilv/libltxhip.so; do
  echo "== bench $L"
  LTX_HIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>>gpurun_out/ab.err | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], [(k["kernel"][:48], round(k["ms_per_step"],2)) for k in d["kernels"][:8]])' || exit $?
done; done
