"""Counter-measured HBM traffic of ONE whole bench step, from the rocprofv3
PMC passes of tools/gpu_step_traffic.sh (bench.py --steps 1 --warmup 1).

Every step ends with check_evolution's k_evolution_final dispatch, so the
dispatches after the first k_evolution_final up to and including the second
are exactly the timed step.  Bytes = FETCH_SIZE x 2 (gfx950: FETCH_SIZE counts
half the bytes of wide coalesced reads, MI355X_MICROARCH.md) + WRITE_SIZE,
summed over those dispatches (FETCH also counts Infinity-Cache hits, so this
is an upper bound on HBM bytes).

Usage: step_traffic.py <dir> <config> <out.json>"""
import collections
import csv
import glob
import json
import re
import sys

d, config, out = sys.argv[1], sys.argv[2], sys.argv[3]


def rows(pattern):
    f = glob.glob(f"{d}/{pattern}", recursive=True)
    if not f:
        sys.exit(f"missing {pattern} under {d}")
    return list(csv.DictReader(open(f[0])))


def short(name):
    m = re.search(r"k_\w+(<[^>]*>)?", name)
    return m.group(0) if m else name[:40]


def per_dispatch(pattern, cname):
    """[(dispatch id, kernel, value kB)] in dispatch order"""
    acc = {}
    for r in rows(pattern):
        if r["Counter_Name"] != cname:
            continue
        key = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        k, v = acc.get(key, (short(r["Kernel_Name"]), 0.0))
        acc[key] = (k, v + float(r["Counter_Value"]))
    return [(i, *acc[i]) for i in sorted(acc)]


def one_step(seq):
    ends = [n for n, (_, k, _) in enumerate(seq) if k == "k_evolution_final"]
    if len(ends) < 2:
        sys.exit(f"need two k_evolution_final dispatches, found {len(ends)}")
    return seq[ends[0] + 1: ends[1] + 1]


fetch = one_step(per_dispatch("pmc_fetch/**/*counter_collection.csv", "FETCH_SIZE"))
write = one_step(per_dispatch("pmc_write/**/*counter_collection.csv", "WRITE_SIZE"))
if len(fetch) != len(write):
    sys.exit(f"the two passes saw different dispatch counts ({len(fetch)} vs {len(write)})")
by_kernel = collections.defaultdict(lambda: [0, 0.0, 0.0])
for (_, k, f), (_, k2, w) in zip(fetch, write):
    if k != k2:
        sys.exit(f"dispatch order differs between passes: {k} vs {k2}")
    e = by_kernel[k]
    e[0] += 1
    e[1] += 2 * f * 1024
    e[2] += w * 1024
fb = sum(e[1] for e in by_kernel.values())
wb = sum(e[2] for e in by_kernel.values())
res = {
    "config": config,
    "dispatches_per_step": len(fetch),
    "bytes_per_step": fb + wb,
    "fetch_bytes_x2": fb,
    "write_bytes": wb,
    "correction": "FETCH_SIZE x 2 x 1024 (gfx950, MI355X_MICROARCH.md) + WRITE_SIZE x 1024; FETCH includes "
                  "Infinity-Cache hits (upper bound on HBM bytes)",
    "kernels": {k: {"dispatches": e[0], "bytes": e[1] + e[2]}
                for k, e in sorted(by_kernel.items(), key=lambda kv: -(kv[1][1] + kv[1][2]))},
}
with open(out, "w") as f:
    json.dump(res, f, indent=1)
print(f"{config}: {len(fetch)} dispatches, {(fb + wb) / 1e9:.3f} GB per step")
