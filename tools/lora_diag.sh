R=$GRAFT_REPO_ROOT; cd /tmp; export TMPDIR=/tmp
for d in 0 1 2 4 7; do
  if [ $d = 0 ]; then L=libltxhip.so; else L=libltxhip_ld$d.so; fi
  LTX_HIP_LIB=$R/video-generation-for-human-avatars_amd/ltx_amd/$L timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ld_$d -o run -- python3 $R/tools/lora_ab.py > /dev/null 2>&1 || exit $?
  python3 -c "
import csv
for r in csv.DictReader(open('/tmp/ld_$d/run_kernel_stats.csv')):
    if 'lora_dy' in r['Name']: print('diag $d', r['Name'][:40], r['Calls'], r['AverageNs'])"
done
