# Round 5: kernel arguments preloaded into SGPRs (-mllvm
# -amdgpu-kernarg-preload-count=16, variant kpre in _lib/ab/: 29 of 75 kernels,
# those with scalar arguments) vs the in-tree library, C0 twice, C1 once.
set -o pipefail
cd $GRAFT_REPO_ROOT
CFG=c0 bash tools/gpu_ab_prof.sh base kpre > gpurun_out/ab_kpre_c0.txt 2>&1 || { tail -20 gpurun_out/ab_kpre_c0.txt; exit 1; }
head -20 gpurun_out/ab_kpre_c0.txt
CFG=c0 bash tools/gpu_ab_prof.sh kpre base > gpurun_out/ab_kpre2_c0.txt 2>&1 || { tail -20 gpurun_out/ab_kpre2_c0.txt; exit 1; }
head -3 gpurun_out/ab_kpre2_c0.txt
CFG=c1 bash tools/gpu_ab_prof.sh base kpre > gpurun_out/ab_kpre_c1.txt 2>&1 || { tail -20 gpurun_out/ab_kpre_c1.txt; exit 1; }
head -12 gpurun_out/ab_kpre_c1.txt
