"""Summaries from a rocprofv3 rocpd database (results.db): per-kernel launch
counts and average / total durations, and a timeline window of kernel
dispatches (start offsets, durations, queue) to see the gaps between them.

    python3 profiles/rocpd_summary.py DB [--timeline N] [--skip S] [--kernel SUBSTR]
                                         [--window-kernel NAME --window N]

--window-kernel / --window: only the dispatches between the start of NAME's
N-th last dispatch and the end of its last one (e.g. the bench's per-kernel
timing window: its last `steps` ticks, 10 k_forces_couple launches a tick)."""
import argparse
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--timeline", type=int, default=0, help="print N consecutive dispatches")
ap.add_argument("--skip", type=int, default=0, help="... starting at dispatch S (time order)")
ap.add_argument("--kernel", default=None, help="only kernels whose name contains this")
ap.add_argument("--api", type=int, default=0, help="also the N host API calls (HIP / RCCL regions) of most total time")
ap.add_argument("--window-kernel", default=None, help="restrict to a window of this kernel's last dispatches")
ap.add_argument("--window", type=int, default=0, help="... its last N dispatches")
ap.add_argument("--json", default=None, help="also write {kernel: {calls, avg_us}} + _build (the library's sha256) here")
ap.add_argument("--lib", default="little-physics-engine_amd/liblpe_hip.so", help="the library profiled (--json stamp)")
a = ap.parse_args()
c = sqlite3.connect(a.db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
if "queue_id" in cols:
    rows = c.execute(f"select {name_col}, start, end, queue_id from kernels order by start").fetchall()
else:
    rows = [(n, s, e, 0) for n, s, e in c.execute(f"select {name_col}, start, end from kernels order by start")]
if a.window_kernel and a.window > 0:
    mine = [r for r in rows if a.window_kernel in r[0]]
    if len(mine) >= a.window:
        w0, w1 = mine[-a.window][1], mine[-1][2]
        rows = [r for r in rows if r[1] >= w0 and r[2] <= w1]
        print(f"window: the last {a.window} dispatches of {a.window_kernel}, {(w1 - w0) / 1e3:.1f} us")
if a.kernel:
    rows = [r for r in rows if a.kernel in r[0]]
agg = {}
for n, s, e, q in rows:
    short = n.split("(")[0].split("<")[0].replace("void ", "").replace("lpe::", "")
    d = agg.setdefault(short, [0, 0.0])
    d[0] += 1
    d[1] += (e - s) / 1e3
tot = sum(v[1] for v in agg.values())
print(f"{'kernel':40s} {'calls':>7s} {'avg us':>9s} {'total us':>11s} {'%':>6s}")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{k[:40]:40s} {n:7d} {t / n:9.2f} {t:11.1f} {100 * t / tot:6.2f}")
if a.json:
    import hashlib
    import json
    out = {k: dict(calls=n, avg_us=round(t / n, 3)) for k, (n, t) in agg.items()}
    out["_build"] = dict(lib_sha256=hashlib.sha256(open(a.lib, "rb").read()).hexdigest(),
                         window=f"last {a.window} dispatches of {a.window_kernel}" if a.window_kernel else "all")
    json.dump(out, open(a.json, "w"), indent=1)
if rows:
    span = (rows[-1][2] - rows[0][1]) / 1e3
    print(f"dispatches {len(rows)}, span {span:.1f} us, kernel time {tot:.1f} us")
if a.api:
    reg = c.execute("select name, count(*), sum(end - start) from regions group by name order by 3 desc limit ?",
                    (a.api,)).fetchall()
    print(f"{'host API':40s} {'calls':>7s} {'avg us':>9s} {'total us':>11s}")
    for n, k, t in reg:
        print(f"{n[:40]:40s} {k:7d} {t / 1e3 / k:9.2f} {t / 1e3:11.1f}")
if a.timeline:
    a.skip = max(0, min(a.skip, len(rows) - a.timeline))
    t0 = rows[a.skip][1]
    prev_end = None
    for n, s, e, q in rows[a.skip:a.skip + a.timeline]:
        short = n.split("(")[0].split("<")[0].replace("void ", "").replace("lpe::", "")
        gap = "" if prev_end is None else f"{(s - prev_end) / 1e3:8.2f}"
        print(f"{(s - t0) / 1e3:10.2f} {(e - s) / 1e3:8.2f} {gap:>8s} q{q} {short[:50]}")
        prev_end = e if prev_end is None else max(prev_end, e)
