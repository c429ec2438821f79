"""One tick of a rocprofv3 kernel trace as a listing: start offset, duration, queue, kernel.

    python profiles/tick_gantt.py KERNEL_TRACE.csv [--tick N] [--marker k_gather_rigids]

Ticks are delimited by the marker kernel (see timeline.py); N counts back from the last
marker (default 40). Gaps where no kernel runs are printed as '-- idle --' lines.
"""
import csv
import re
import sys


def main():
    src = sys.argv[1]
    back = int(sys.argv[sys.argv.index("--tick") + 1]) if "--tick" in sys.argv else 40
    marker = sys.argv[sys.argv.index("--marker") + 1] if "--marker" in sys.argv else "k_gather_rigids"
    rows = []
    for r in csv.DictReader(open(src)):
        name = r.get("Kernel_Name") or ""
        m = re.match(r"(?:void )?(?:lpe::)?([A-Za-z_][\w]*)", name)
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else name, q))
    rows.sort()
    marks = [a for a, b, k, q in rows if k == marker]
    lo, hi = marks[-back - 1], marks[-back]
    busy_until = lo
    for a, b, k, q in rows:
        if a < lo or a >= hi:
            continue
        if a > busy_until + 2000:
            print(f"{(busy_until - lo) / 1e3:9.1f}  -- idle {(a - busy_until) / 1e3:.1f} us --")
        print(f"{(a - lo) / 1e3:9.1f} {(b - a) / 1e3:8.1f}  q{q:>3}  {k}")
        busy_until = max(busy_until, b)
    print(f"tick {(hi - lo) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
