# C4 rehearsal on ONE GPU: 8 in-process ranks x 10 M cells (80 M cells), the
# whole distributed algorithm (global AMG hierarchy built on every rank's
# host, segment all-gathers, halos) with the peer-copy transport.  A
# heartbeat line every minute keeps the long setup visibly alive.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while true; do sleep 60; echo "[heartbeat] $(date +%T)"; done ) &
HB=$!
CFD_AMG_TIMING=1 timeout -k 10 1000 python -u bench.py --config c2 --inproc-ranks 8 --steps 2 --warmup 1 \
  --no-cpu-baseline --ref-workloads 0 > gpurun_out/inproc8_c4.json 2> gpurun_out/inproc8_c4.log
rc=$?
kill $HB
cut -c1-600 gpurun_out/inproc8_c4.json
tail -20 gpurun_out/inproc8_c4.log
exit $rc
