# Round-5 evidence, part D: C4 as 8 in-process ranks on one GPU (the whole
# distributed algorithm), with the comm-timing table of the extra step -- the
# global hierarchy (default) and the partition-aware mode (--amg-local 1),
# one mesh (cached) for both.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for mode in 0 1; do
  timeout -k 10 900 python -u bench.py --round r05 --inproc-ranks 8 --steps 3 --warmup 2 --ref-workloads 0 --no-cpu-baseline \
    --amg-local $mode --mesh-cache /tmp/c4_inproc8_mesh.bin > gpurun_out/bench_inproc8_local${mode}_r05.json 2> gpurun_out/bench_inproc8_local${mode}_r05.log || exit $?
  python -c "import json; d=json.load(open('gpurun_out/bench_inproc8_local${mode}_r05.json')); c=d['comm']; print('local=$mode', d['ms_per_step'], 'ms/step; exchanges/it', c['exchanges_per_iteration'], 'allgathers/it', c['allgathers_per_iteration'], 'halo B/it', c['halo_bytes_per_iteration'])"
done
