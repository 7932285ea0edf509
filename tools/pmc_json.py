"""Per-kernel means of rocprofv3 --pmc counter collections -> one JSON file.

    python tools/pmc_json.py waits OUT.json DIR...   # SQ / SQC wait + icache split
    python tools/pmc_json.py ta OUT.json DIR...      # texture-addresser issue load

Each DIR holds one pass's *_counter_collection.csv (gpurun_out/pmc_ic_r06/sq,
gpurun_out/r06_ta_after/ta ...).  Values are per-dispatch medians over the
launches of each kernel (short name: template arguments kept, parameter list
dropped), then the derived fractions the DESIGN tables quote.
"""
import csv
import glob
import json
import statistics
import sys
from collections import defaultdict


def short(name):
    for p in ("void ", "rlmd::", "(anonymous namespace)::"):
        name = name.replace(p, "")
    depth = 0
    for i, ch in enumerate(name):
        depth += (ch == "<") - (ch == ">")
        if ch == "(" and depth == 0:
            return name[:i]
    return name


def collect(dirs):
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> dispatch -> value
    for d in dirs:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                per[short(r["Kernel_Name"])][r["Counter_Name"]][r["Dispatch_Id"]] = float(r["Counter_Value"])
    out = {}
    for k, cs in per.items():
        row = {"dispatches": max(len(v) for v in cs.values())}
        for c, v in sorted(cs.items()):
            row[c] = statistics.median(v.values())
        out[k] = row
    return out


def derive_waits(row):
    cyc = row.get("SQ_WAVE_CYCLES")
    if cyc:
        w, wi, act = row.get("SQ_WAIT_ANY", 0), row.get("SQ_WAIT_INST_ANY", 0), row.get("SQ_ACTIVE_INST_ANY", 0)
        row["frac_waitcnt"] = w / cyc
        row["frac_issue_wait"] = wi / cyc
        row["frac_active"] = act / cyc
    h, m = row.get("SQC_ICACHE_HITS"), row.get("SQC_ICACHE_MISSES")
    if h is not None and m is not None and h + m:
        row["icache_miss_rate"] = m / (h + m)


def derive_ta(row):
    waves, buf, busy = row.get("SQ_WAVES"), row.get("TA_BUFFER_WAVEFRONTS"), row.get("TA_TA_BUSY")
    if waves:
        row["buffer_instr_per_wave"] = buf / waves if buf is not None else None
    row["ta_cycles_per_buffer_instr"] = busy / buf if buf else None


def main():
    kind, out, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    rows = collect(dirs)
    for row in rows.values():
        (derive_waits if kind == "waits" else derive_ta)(row)
    meta = {"source": dirs, "method": "per-kernel medians over dispatches of each counter; SQ_* summed over the chip"}
    if kind == "waits":
        meta["fractions"] = ("frac_waitcnt = SQ_WAIT_ANY / SQ_WAVE_CYCLES; frac_issue_wait = "
                             "SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES; frac_active = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES")
    json.dump({"meta": meta, "kernels": rows}, open(out, "w"), indent=1, sort_keys=False)
    for k, r in rows.items():
        print(k[:70], {c: (round(v, 3) if isinstance(v, float) else v) for c, v in r.items() if c.islower() or c == "dispatches"})


if __name__ == "__main__":
    main()
