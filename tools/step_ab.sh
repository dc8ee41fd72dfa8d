# interleaved whole-step A/B in one GPU call: tools/step_ab.sh "ENV=a ENV2=b" "ENV=c" [rounds]
# (bench.py --steps 12 --warmup 3, one JSON line per run into gpurun_out/step_ab.jsonl)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
A=$1; B=$2; N=${3:-2}
: > gpurun_out/step_ab.jsonl
for i in $(seq 1 $N); do for cfg in "$A" "$B"; do
  echo "== $cfg" | tee -a gpurun_out/step_ab.jsonl
  env $cfg timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/step_ab_one.json 2>/dev/null || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/step_ab_one.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" | tee -a gpurun_out/step_ab.jsonl
done; done
