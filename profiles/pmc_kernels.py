"""Per-kernel means of rocprofv3 --pmc counters (SQ_* and friends) over the
last N dispatches of each kernel.

    python profiles/pmc_kernels.py COUNTER_COLLECTION.csv [--last N] [--kernels a,b,...]

SQ_WAVE_CYCLES / SQ_BUSY_CYCLES and the SQ_WAIT_* counters count quad-cycles
on gfx950 (MI355X_MICROARCH.md, constants table); SQ_INSTS_* count wave
instructions.
"""
import csv
import json
import re
import sys
from collections import defaultdict


def main():
    src = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 50
    only = sys.argv[sys.argv.index("--kernels") + 1].split(",") if "--kernels" in sys.argv else None
    vals = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(src)):
        m = re.match(r"(?:void )?(?:lpe::)?(\w+)", r["Kernel_Name"])
        k = m.group(1)
        if only and k not in only:
            continue
        vals[k][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out = {}
    for k, cs in vals.items():
        out[k] = {}
        for c, v in cs.items():
            v.sort()
            tail = [x for _, x in v[-last:]]
            out[k][c] = sum(tail) / len(tail)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
