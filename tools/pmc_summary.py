"""Turn one round's rocprofv3 outputs (tools/profile_round.sh) into profiles/:

writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, per kernel),
profiles/<tag>_kernel_summary.txt (top kernels, per-dispatch averages) and
profiles/<tag>_pmc_env.json: HBM bytes per launch of the env step from the
separate FETCH_SIZE and WRITE_SIZE passes (the fused act_env_kernel minus the
acting kernel when the trace has both, else env_train_kernel), tagged with
"kernel_id", "round" and "config" so that bench.py attaches it only to the
roofline of the same kernel and workload.

  python tools/pmc_summary.py r03 [c2]

Units and gfx950 corrections (MI355X_MICROARCH.md, HBM section): both counters are KiB; FETCH_SIZE counts
half the bytes of wide coalesced reads on gfx950, so it is doubled.
"""
import csv
import re
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter(path, name, kernel="env_train_kernel"):
    vals, grids = [], set()
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == name:
                vals.append(float(row["Counter_Value"]))
                grids.add(int(row["Grid_Size"]))
    return vals, grids


def mfma_summary(path, stat_rows, dst):
    """MFMA utilisation per learn / acting kernel from one --pmc pass:
    SQ_VALU_MFMA_BUSY_CYCLES (cycles a SIMD's MFMA pipe is busy, summed over the
    chip) / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): the fraction of the chip's
    MFMA pipe-cycles used while the kernel ran."""
    per = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            m = re.search(r"(\w+_kernel)", row["Kernel_Name"])
            k = m.group(1) if m else row["Kernel_Name"][:60]
            d = per.setdefault(k, {}).setdefault(row["Dispatch_Id"], {})
            d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    out = {}
    for k, ds in per.items():
        busy = statistics.median(d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for d in ds.values())
        gui = statistics.median(d.get("GRBM_GUI_ACTIVE", 0.0) for d in ds.values())
        sq = statistics.median(d.get("SQ_BUSY_CYCLES", 0.0) for d in ds.values())
        out[k] = {"dispatches": len(ds), "mfma_busy_cycles": busy, "grbm_gui_active": gui, "sq_busy_cycles": sq,
                  "mfma_util": busy / (gui / 8.0 * 1024.0) if gui else None}
    out["_method"] = ("medians over dispatches; mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 "
                      "SIMDs); GRBM_GUI_ACTIVE is summed over the 8 XCDs by rocprofv3 (MI355X_MICROARCH.md)")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


def trace_roofline(path, lanes=65536, bytes_per_lane=103):
    """The headline roofline recomputed from the per-dispatch kernel trace of the
    same bench command, as bench.py computes it live: act_env_kernel's average
    full-size dispatch minus the acting-only kernel's inside whole unfused train
    steps (fused_act_kernel dispatches directly followed by env_train_kernel: the
    same cache state, after the previous step's updates), against 103 B x lanes.
    The back-to-back acting-only launches (bench.py's 20 reference launches) are
    reported beside; 100-row evaluation launches are excluded (grid = 4 x lanes)."""
    rows = []
    with open(path) as f:
        for row in csv.DictReader(f):
            m = re.search(r"(\w+_kernel)", row["Kernel_Name"])
            rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), m.group(1) if m else "",
                         int(row["Grid_Size_X"])))
    rows.sort()
    fused, in_step, b2b = [], [], []
    for i, (t0, t1, k, g) in enumerate(rows):
        if g != 4 * lanes:
            continue
        if k == "act_env_kernel":
            fused.append((t1 - t0) * 1e-3)
        elif k == "fused_act_kernel":
            nxt = rows[i + 1][2] if i + 1 < len(rows) else ""
            (in_step if nxt == "env_train_kernel" else b2b).append((t1 - t0) * 1e-3)
    if not fused or not in_step:
        return None
    fa, act = statistics.median(fused), statistics.median(in_step)
    marg = fa - act
    gbs = bytes_per_lane * lanes / (marg * 1e-6) / 1e9
    return {"act_env_us": fa, "act_env_mean_us": statistics.mean(fused), "act_env_launches": len(fused),
            "fused_act_in_step_us": act, "fused_act_in_step_mean_us": statistics.mean(in_step),
            "fused_act_in_step_launches": len(in_step),
            "fused_act_back_to_back_us": statistics.median(b2b) if b2b else None, "marginal_us": marg,
            "algorithmic_bytes_per_launch": bytes_per_lane * lanes, "achieved_GBs": gbs, "frac": gbs / 8000.0,
            "method": f"medians over dispatches with grid {4 * lanes} work-items (as bench.py's live samples); "
                      "acting-only = fused_act_kernel dispatches followed by env_train_kernel (in whole unfused steps)"}


def main(tag, config="c2"):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"rocprofv3 --kernel-trace --stats: python bench.py --no-cpu-baseline --no-companion --k-sweep= "
             f"--seeds-per-gpu= --seed-procs= --steps 25 --warmup 5 "
             f"(C2, 65,536 GBM lanes, SAC 256/256 bf16, K=8)", "",
             f"{'calls':>6} {'avg_us':>9} {'total_ms':>9} {'pct':>6}  kernel"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        n, t = int(r["Calls"]), float(r["TotalDurationNs"])
        lines.append(f"{n:6d} {t / n / 1e3:9.2f} {t / 1e6:9.3f} {100 * t / tot:6.2f}  {r['Name'][:120]}")
    tpath = os.path.join(src, "trace", "trace_kernel_trace.csv")
    roof = trace_roofline(tpath) if config == "c2" and os.path.exists(tpath) else None
    if roof:
        lines += ["", "headline roofline from this trace (act_env_kernel - fused_act_kernel, full-size launches):",
                  json.dumps(roof)]
        json.dump(roof, open(os.path.join(dst, f"{tag}_roofline_trace.json"), "w"), indent=1)
    open(os.path.join(dst, f"{tag}_kernel_summary.txt"), "w").write("\n".join(lines) + "\n")
    fpath = os.path.join(src, "fetch", "fetch_counter_collection.csv")
    wpath = os.path.join(src, "write", "write_counter_collection.csv")
    per = {}
    for k in ("act_env_kernel", "fused_act_kernel", "env_train_kernel"):
        fetch, g1 = counter(fpath, "FETCH_SIZE", k)
        write, g2 = counter(wpath, "WRITE_SIZE", k)
        if fetch and write:
            per[k] = {"launches": [len(fetch), len(write)], "grid": sorted(g1 | g2)[0],
                      "fetch_bytes": 2.0 * 1024.0 * statistics.median(fetch),
                      "write_bytes": 1024.0 * statistics.median(write)}
            per[k]["hbm_bytes"] = per[k]["fetch_bytes"] + per[k]["write_bytes"]
    if "act_env_kernel" in per and "fused_act_kernel" in per:
        a, b = per["act_env_kernel"], per["fused_act_kernel"]
        out = {"kernel": "act_env_kernel - fused_act_kernel (the env step's marginal traffic)",
               "kernel_id": "act_env_marginal",
               "lanes": a["grid"] // 4, "hbm_bytes_per_launch": a["hbm_bytes"] - b["hbm_bytes"],
               "fetch_bytes_per_launch": a["fetch_bytes"] - b["fetch_bytes"],
               "write_bytes_per_launch": a["write_bytes"] - b["write_bytes"], "per_kernel": per}
    else:
        e = per["env_train_kernel"]
        out = {"kernel": "env_train_kernel", "kernel_id": "env_train_kernel", "lanes": e["grid"], "launches": e["launches"],
               "fetch_bytes_per_launch": e["fetch_bytes"], "write_bytes_per_launch": e["write_bytes"],
               "hbm_bytes_per_launch": e["hbm_bytes"], "per_kernel": per}
    out["round"], out["config"] = tag, config
    out["method"] = ("median over launches of separate --pmc FETCH_SIZE / --pmc WRITE_SIZE passes; KiB x 1024; "
                     "FETCH_SIZE doubled (gfx950 half-count of wide coalesced reads)")
    json.dump(out, open(os.path.join(dst, f"{tag}_pmc_env.json"), "w"), indent=1)
    mf = os.path.join(src, "mfma", "mfma_counter_collection.csv")
    if os.path.exists(mf):
        mfma_summary(mf, rows, os.path.join(dst, f"{tag}_pmc_mfma.json"))
    print(json.dumps(out, indent=1))
    print("\n".join(lines[:14]))


CONFIG_NAMES = {"c3": "C3, 65,536 Dice_SH_InvA lanes, TD3 400/300 bf16, B = 200, K = 8",
                "c4": "C4, 8,192 Market_InvA_D1 lanes on stooq_snp, SAC 256/256 bf16, K = 8",
                "c5": "C5, 65,536 GBM_InvA lanes, TD3 400/300 bf16, 5-step returns, 2^24-row ring, K = 8"}
LEARN = ("fwd_rows_kernel", "critic_update_kernel", "qeval_rows_kernel", "actor_update_kernel")


def config_summaries(tag):
    """profiles/<tag>_<cfg>_kernel_summary.txt (+ _pmc_mfma.json) for the C3 / C4 / C5
    traces of tools/gpu_prof_configs.sh (headline region only: no seed groups or
    variants), with the learner's time per update (launch counts weight the TD3
    kernels that run every second update)."""
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    for cfg, name in CONFIG_NAMES.items():
        stats = os.path.join(src, f"trace_{cfg}", "trace_kernel_stats.csv")
        if not os.path.exists(stats):
            continue
        rows = list(csv.DictReader(open(stats)))
        tot = sum(float(r["TotalDurationNs"]) for r in rows)
        lines = [f"rocprofv3 --kernel-trace --stats: python bench.py --config {cfg} --no-cpu-baseline --no-companion "
                 f"--k-sweep= --seeds-per-gpu= --seed-procs= --variants= --steps 25 --warmup 5 ({name})", "",
                 f"{'calls':>6} {'avg_us':>9} {'total_ms':>9} {'pct':>6}  kernel"]
        per_kernel = {}
        for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
            n, t = int(r["Calls"]), float(r["TotalDurationNs"])
            lines.append(f"{n:6d} {t / n / 1e3:9.2f} {t / 1e6:9.3f} {100 * t / tot:6.2f}  {r['Name'][:120]}")
            m = re.search(r"(\w+_kernel)", r["Name"])
            if m and m.group(1) in LEARN:
                c, tt = per_kernel.get(m.group(1), (0, 0.0))
                per_kernel[m.group(1)] = (c + n, tt + t)
        if "critic_update_kernel" in per_kernel:
            n_upd = per_kernel["critic_update_kernel"][0]  # one critic step per update
            per_upd = sum(t for _, t in per_kernel.values()) / n_upd / 1e3
            lines += ["", f"learner time per update: {per_upd:.2f} us over {n_upd} updates "
                          "(sum of the four learner kernels' total time / critic steps)"]
        open(os.path.join(ROOT, "profiles", f"{tag}_{cfg}_kernel_summary.txt"), "w").write("\n".join(lines) + "\n")
        print("\n".join(lines[:10] + lines[-1:]))
        mf = os.path.join(src, f"mfma_{cfg}", "mfma_counter_collection.csv")
        if os.path.exists(mf):
            mfma_summary(mf, rows, os.path.join(ROOT, "profiles", f"{tag}_{cfg}_pmc_mfma.json"))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "configs":
        config_summaries(sys.argv[1])
    else:
        main(sys.argv[1] if len(sys.argv) > 1 else "r01", sys.argv[2] if len(sys.argv) > 2 else "c2")
