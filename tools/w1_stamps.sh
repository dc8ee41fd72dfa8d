# phase stamps of the one-wave backward kernels (diag library); args: dkdv mode, dq mode (12 / 22)
export LTX_HIP_LIB=$GRAFT_REPO_ROOT/video-generation-for-human-avatars_amd/ltx_amd/libltxhip_diag.so
timeout -k 10 120 python -u tools/dkdv_stamps.py ${1:-12} > gpurun_out/st_dkdv.txt 2>&1 && timeout -k 10 120 python -u tools/dq_stamps.py ${2:-12} > gpurun_out/st_dq.txt 2>&1
