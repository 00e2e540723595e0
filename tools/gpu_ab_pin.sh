# GPU tests on the product library, then same-box A/B of the reference's two
# benchmarks (natural convergence) for library variants $VARIANTS.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -2 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -30; exit $rc; fi
for v in ${VARIANTS:-new pin new pin}; do
  CFD2_AMD_LIB=$PWD/cfd-demo2_amd/cfd2_amd/_lib/ab/libcfd2_amd_$v.so timeout -k 10 300 python -u tools/ref_workload_run.py all > gpurun_out/ab_pin_$v.json 2> gpurun_out/ab_pin_$v.log || exit $?
  python -c "
import json; d=json.load(open('gpurun_out/ab_pin_$v.json'))
print('$v', {k: round(x['ms_per_step'], 3) for k, x in d.items()})"
done
