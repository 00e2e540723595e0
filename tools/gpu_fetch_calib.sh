# FETCH_SIZE / WRITE_SIZE calibration per access width (tools/fetch_calib.hip):
# one rocprofv3 pass per counter, each under its own time limit.
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/fetch_calib
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $ROOT/tools/bin/fetch_calib > $OUT/fetch.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $ROOT/tools/bin/fetch_calib > $OUT/write.log 2>&1 && \
python3 - "$OUT" <<'PY'
import csv, glob, sys, re
d = sys.argv[1]
for cname, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
    f = glob.glob(f"{d}/{sub}/**/*counter_collection.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == cname]
    acc = {}
    for r in rows:
        k = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        n, v = acc.get(k, (r["Kernel_Name"], 0.0))
        acc[k] = (n, v + float(r["Counter_Value"]))
    for k in sorted(acc)[4:]:  # the second round
        n, v = acc[k]
        print(f"{cname:10s} {re.sub(r'[(].*', '', n)[:24]:24s} {v * 1024 / 2**30:8.3f} x 2^30 bytes (counter kB x 1024 / 1 GiB)")
PY
