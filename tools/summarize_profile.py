#!/usr/bin/env python
"""Summarise a tools/gpu_profile.sh run (gpurun_out/prof/*) into profiles/<tag>_summary.json and
copy the rocprofv3 --stats table next to it.

Per kernel: average duration (kernel-trace), FETCH_SIZE / WRITE_SIZE per dispatch (KB as reported
by rocprofv3), HBM traffic corrected with the calibration kernels of tools/calib_fetch.hip (known
byte counts at 4/8/16 B per lane: on gfx950 FETCH_SIZE reports 1/2 of the bytes read, WRITE_SIZE
all bytes written — MI355X_MICROARCH.md "HBM"), VALU instructions and active cycles per wave,
waves, and the effective clock from GRBM_GUI_ACTIVE.
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mean_counter(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: statistics.mean(v) for k, v in out.items()}


def calibration(prof):
    """bytes / counter-bytes for reads (worst case over 4/8/16 B per lane) and 8-B writes."""
    out = {}
    for counter, kern in (("FETCH_SIZE", ("read4", "read8", "read16")), ("WRITE_SIZE", ("write8",))):
        path = os.path.join(prof, f"calib_{counter}", "run_counter_collection.csv")
        if not os.path.exists(path):
            return None
        per = {}
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0]
            if name in kern and r["Counter_Name"] == counter:
                per.setdefault(name, []).append(float(r["Counter_Value"]) * 1024)
        out[counter] = {k: (512 << 20) / statistics.mean(v) for k, v in per.items()}
    return out


def main(tag, prof=os.path.join(ROOT, "gpurun_out", "prof"), bench_log=None, trace_sweeps=None, pmc_sweeps=None,
         calib=None):
    """trace_sweeps: sweeps of each persist_kernel dispatch of the trace pass, in order (the bench's
    warmup, steps, roofline-pass launches); pmc_sweeps: sweeps of the PMC passes' one persistent
    dispatch.  The persistent kernel runs many sweeps per launch, so its per-dispatch counters are
    divided by these to give per-sweep figures (bench.py does the same)."""
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    stats = list(csv.DictReader(open(os.path.join(prof, "trace", "run_kernel_stats.csv"))))
    shutil.copy(os.path.join(prof, "trace", "run_kernel_stats.csv"), os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    trace = list(csv.DictReader(open(os.path.join(prof, "trace", "run_kernel_trace.csv"))))
    res = {"tag": tag, "kernels": {}}
    cal = calibration(calib or prof)
    if cal:
        res["calibration"] = cal
    f_read = cal["FETCH_SIZE"]["read8"] if cal else 2.0   # guide: FETCH_SIZE = 1/2 of the bytes read
    f_write = cal["WRITE_SIZE"]["write8"] if cal else 1.0
    fetch = mean_counter(os.path.join(prof, "fetch_size", "run_counter_collection.csv"), "FETCH_SIZE")
    write = mean_counter(os.path.join(prof, "write_size", "run_counter_collection.csv"), "WRITE_SIZE")
    vpath = os.path.join(prof, "sq_insts_valu", "run_counter_collection.csv")
    valu = {c: mean_counter(vpath, c) for c in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_WAVES",
                                               "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE")}
    for r in stats:
        name = r["Name"]
        if name.startswith("__amd"):
            continue
        k = dict(calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]), min_ns=float(r["MinNs"]), max_ns=float(r["MaxNs"]),
                 stddev_ns=float(r["StdDev"]))
        rows = [t for t in trace if t["Kernel_Name"] == name]
        if len(rows) > 2:
            st = [int(t["Start_Timestamp"]) for t in rows]
            en = [int(t["End_Timestamp"]) for t in rows]
            k["median_gap_ns"] = statistics.median([st[i + 1] - en[i] for i in range(len(rows) - 1)])
        if "persist_kernel" in name:
            if trace_sweeps and len(trace_sweeps) <= len(rows):
                # the list names the bench's own dispatches, the last ones of the trace; earlier ones
                # are the clock settle's scratch sampler (bench.settle_clocks, round 6), not counted
                if len(rows) > len(trace_sweeps):
                    k["settle_dispatches"] = len(rows) - len(trace_sweeps)
                    rows = rows[len(rows) - len(trace_sweeps):]
                k["dispatches"] = [dict(sweeps=n, ns=int(t["End_Timestamp"]) - int(t["Start_Timestamp"]),
                                        ns_per_sweep=(int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / n)
                                   for n, t in zip(trace_sweeps, rows)]
                k["ns_per_sweep"] = sum(d["ns"] for d in k["dispatches"]) / sum(trace_sweeps)
            if pmc_sweeps:
                k["sweeps_per_dispatch"] = pmc_sweeps  # of the PMC passes (counters below are per dispatch)
        if name in fetch:
            k["fetch_size_kb"] = fetch[name]
        if name in write:
            k["write_size_kb"] = write[name]
        if name in fetch and name in write:
            k["traffic_bytes_uncorrected"] = (fetch[name] + write[name]) * 1024
            k["traffic_bytes"] = (fetch[name] * f_read + write[name] * f_write) * 1024
            k["traffic_correction"] = dict(read=f_read, write=f_write)
            if k.get("sweeps_per_dispatch"):
                k["traffic_bytes_per_sweep"] = k["traffic_bytes"] / k["sweeps_per_dispatch"]
        if name in valu["SQ_WAVES"]:
            waves = valu["SQ_WAVES"][name]
            k["waves"] = waves
            k["valu_insts_per_wave"] = valu["SQ_INSTS_VALU"][name] / waves
            k["valu_active_quadcycles_per_wave"] = valu["SQ_ACTIVE_INST_VALU"][name] / waves
            k["wave_quadcycles_per_wave"] = valu["SQ_WAVE_CYCLES"][name] / waves
            k["valu_active_frac_of_wave_lifetime"] = valu["SQ_ACTIVE_INST_VALU"][name] / valu["SQ_WAVE_CYCLES"][name]
            gui = valu["GRBM_GUI_ACTIVE"][name]
            k["grbm_gui_active"] = gui
        res["kernels"][name] = k
    if bench_log and os.path.exists(bench_log):
        for line in open(bench_log):
            if line.startswith("{"):
                res["bench_line_under_profiler"] = json.loads(line)
    out = os.path.join(ROOT, "profiles", f"{tag}_summary.json")
    json.dump(res, open(out, "w"), indent=1)
    print(out)
    for n, k in res["kernels"].items():
        print(n[:70], {a: (round(b, 3) if isinstance(b, float) else b) for a, b in k.items()})


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--trace-sweeps", default="", help="comma list: sweeps of each persistent dispatch (trace pass)")
    ap.add_argument("--pmc-sweeps", type=int, default=0, help="sweeps of the PMC passes' persistent dispatch")
    ap.add_argument("--prof", default=os.path.join(ROOT, "gpurun_out", "prof"))
    ap.add_argument("--bench-log", default=os.path.join(ROOT, "gpurun_out", "prof_trace.log"))
    ap.add_argument("--calib", default=None, help="directory holding calib_FETCH_SIZE/ calib_WRITE_SIZE/")
    a = ap.parse_args()
    main(a.tag, prof=a.prof, bench_log=a.bench_log,
         trace_sweeps=[int(x) for x in a.trace_sweeps.split(",") if x], pmc_sweeps=a.pmc_sweeps or None,
         calib=a.calib)
