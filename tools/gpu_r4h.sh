cd "${GRAFT_REPO_ROOT}"
NOSQ=1 REPS=3 OUT=r04h VARIANTS="v4 r16" bash tools/gpu_r4e.sh && \
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase_prof.py 131072 16384 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04h/phase.txt
