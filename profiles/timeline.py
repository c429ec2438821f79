"""Per-tick timeline of a rocprofv3 kernel trace of bench.py.

    python profiles/timeline.py KERNEL_TRACE.csv OUT.json [--ticks N] [--skip M] [--marker k_gather_rigids]

rocprofv3 --kernel-trace --output-format csv writes one row per dispatch with
start / end timestamps (ns).  Ticks are delimited by the launches of a marker
kernel that runs once per tick at its start (k_gather_rigids: the fluid's
rigid gather, sim.cpp:160 -> fluid.cpp:304).  For N complete ticks ending M
ticks before the last marker (--skip M: leave out bench.py's second window,
whose launches carry timing events) this reports:

  tick_us        wall time from marker to marker
  busy_us        time at least one kernel runs (union of dispatch intervals)
  idle_us        tick_us - busy_us (launch gaps, host stalls)
  kernels        per kernel: launches per tick, mean duration, and the time
                 during which it is the ONLY kernel running ("exclusive_us":
                 what the tick would save if it vanished, to first order)

Per-kernel mean durations here are the ones the bench's HIP-event averages
must agree with (same dispatches).
"""
import csv
import json
import re
import sys
from collections import defaultdict


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or ""
            m = re.match(r"(?:void )?(?:lpe::)?([A-Za-z_][\w]*)", name)
            k = m.group(1) if m else name
            t0 = int(r.get("Start_Timestamp") or r.get("BeginNs"))
            t1 = int(r.get("End_Timestamp") or r.get("EndNs"))
            rows.append((t0, t1, k))
    rows.sort()
    return rows


def union_len(iv):
    tot, cur0, cur1 = 0, None, None
    for a, b in sorted(iv):
        if cur0 is None or a > cur1:
            if cur0 is not None:
                tot += cur1 - cur0
            cur0, cur1 = a, b
        else:
            cur1 = max(cur1, b)
    if cur0 is not None:
        tot += cur1 - cur0
    return tot


def exclusive(rows, lo, hi):
    """ns during which each kernel is the only one running, within [lo, hi)."""
    ev = []
    for i, (a, b, k) in enumerate(rows):
        a, b = max(a, lo), min(b, hi)
        if b > a:
            ev.append((a, 1, i))
            ev.append((b, -1, i))
    ev.sort()
    active = set()
    out = defaultdict(int)
    last = None
    for t, d, i in ev:
        if last is not None and len(active) == 1:
            out[rows[next(iter(active))][2]] += t - last
        if d > 0:
            active.add(i)
        else:
            active.discard(i)
        last = t
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    nt = int(sys.argv[sys.argv.index("--ticks") + 1]) if "--ticks" in sys.argv else 10
    marker = sys.argv[sys.argv.index("--marker") + 1] if "--marker" in sys.argv else "k_gather_rigids"
    rows = load(src)
    marks = [a for a, b, k in rows if k == marker]
    if len(marks) < 2:
        raise SystemExit(f"fewer than 2 {marker} launches")
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
    if skip:
        marks = marks[:-skip]
    marks = marks[-(nt + 1):]
    lo, hi = marks[0], marks[-1]
    ticks = len(marks) - 1
    win = [r for r in rows if r[0] >= lo and r[0] < hi]
    busy = union_len([(max(a, lo), min(b, hi)) for a, b, k in win])
    per = defaultdict(list)
    for a, b, k in win:
        per[k].append(b - a)
    exc = exclusive(win, lo, hi)
    kern = {k: {"launches_per_tick": round(len(v) / ticks, 2), "avg_us": round(sum(v) / len(v) / 1e3, 2),
                "total_us_per_tick": round(sum(v) / ticks / 1e3, 1),
                "exclusive_us_per_tick": round(exc.get(k, 0) / ticks / 1e3, 1)}
            for k, v in per.items()}
    kern = dict(sorted(kern.items(), key=lambda kv: -kv[1]["total_us_per_tick"]))
    out = {"what": f"rocprofv3 kernel trace, last {ticks} ticks (marker {marker})",
           "tick_us": round((hi - lo) / ticks / 1e3, 1), "busy_us": round(busy / ticks / 1e3, 1),
           "idle_us": round((hi - lo - busy) / ticks / 1e3, 1), "kernels": kern}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("tick_us", "busy_us", "idle_us")}))
    for k, v in list(kern.items())[:25]:
        print(f"{k:28s} {v['launches_per_tick']:6.1f}/tick {v['avg_us']:8.2f} us  tot {v['total_us_per_tick']:8.1f}"
              f"  excl {v['exclusive_us_per_tick']:8.1f}")


if __name__ == "__main__":
    main()
