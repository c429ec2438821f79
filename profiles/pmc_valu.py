"""VALU / SALU / LDS / VMEM instruction counts per launch from one rocprofv3 SQ pass.

    python profiles/pmc_valu.py SQ.csv OUT.json [--last N]

The pass is `rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES` (8 SQ counters,
one pass).  SQ_INSTS_* count wave instructions (whole chip, per dispatch);
per kernel the mean over its last N dispatches (the timed window at the end of
bench.py) is written; bench.py reports valu_wave_insts as the roofline's
compute side.
"""
import csv
import json
import re
import hashlib
import sys
from collections import defaultdict

FIELDS = {"SQ_INSTS_VALU": "valu_wave_insts", "SQ_INSTS_SALU": "salu_insts", "SQ_INSTS_LDS": "lds_insts",
          "SQ_INSTS_VMEM_RD": "vmem_rd_insts", "SQ_INSTS_VMEM_WR": "vmem_wr_insts", "SQ_WAVES": "waves",
          "SQ_BUSY_CYCLES": "sq_busy_quad_cycles", "SQ_WAVE_CYCLES": "sq_wave_quad_cycles"}


def main():
    src, dst = sys.argv[1:3]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 50
    vals = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(src)):
        c = r["Counter_Name"]
        if c not in FIELDS:
            continue
        k = re.match(r"(?:void )?(?:lpe::)?(\w+)", r["Kernel_Name"]).group(1)
        vals[k][c].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out = {}
    for k, cs in sorted(vals.items()):
        out[k] = {}
        n = None
        for c, v in cs.items():
            v.sort()
            tail = [x for _, x in v[-last:]]
            out[k][FIELDS[c]] = round(sum(tail) / len(tail), 1)
            n = len(tail) if n is None else min(n, len(tail))
        out[k]["dispatches"] = n
        out[k]["method"] = ("rocprofv3 --pmc " + " ".join(FIELDS) + " (one pass), last dispatches of "
                            "bench.py's timed window")
    if "--lib" in sys.argv:     # the library the passes profiled (bench.py compares it with its own)
        lib = sys.argv[sys.argv.index("--lib") + 1]
        out["_build"] = {"lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(), "lib": lib}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
