# Round 4: prepare / assemble with the first faces' loads issued up front
# (in-tree library) against the previous sources (_lib/ab/libcfd2_amd_old.so);
# the kernel-buffer parity tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_tests.sh faces tests/test_gpu_parity.py tests/test_voronoi.py || exit $?
CFG=c2 STEPS=10 bash tools/gpu_ab_prof.sh old base > gpurun_out/ab_faces_c2.txt 2>&1 || exit $?
head -30 gpurun_out/ab_faces_c2.txt
