"""Assemble the density microbench's PMC passes into one summary.

    python profiles/pmc_density.py DIR OUT.json US_PAIR US_PLAN [--lib LIB]

DIR holds D_sq1 / D_sq2 / D_fetch / D_write _counter_collection.csv from
profiles/pmc_collect.sh (rocprofv3 over profiles/density_micro.py --reps 3);
US_*: the launches' average durations from the same build (HIP events)."""
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def kernels(csv, last=3):
    out = subprocess.check_output([sys.executable, os.path.join(HERE, "pmc_kernels.py"), csv, "--last", str(last),
                                   "--kernels", "k_density_pair,k_density_plan"])
    return json.loads(out)


def main():
    d, dst, us_pair, us_plan = sys.argv[1], sys.argv[2], float(sys.argv[3]), float(sys.argv[4])
    d1 = kernels(os.path.join(d, "D_sq1_counter_collection.csv"))
    d2 = kernels(os.path.join(d, "D_sq2_counter_collection.csv"))
    tr = subprocess.check_output([sys.executable, os.path.join(HERE, "pmc_traffic.py"),
                                  os.path.join(d, "D_fetch_counter_collection.csv"),
                                  os.path.join(d, "D_write_counter_collection.csv"), "/tmp/_dt.json", "--last", "3"])
    dt = json.load(open("/tmp/_dt.json"))
    out = {"what": "rocprofv3 --pmc passes (profiles/pmc_collect.sh, one counter group per run) over "
                   "profiles/density_micro.py --reps 3: the 16.7M-particle lattice, the shipped pure density pass "
                   "(k_density_plan + k_density_pair), means over the last 3 launches.  SQ_*_CYCLES / SQ_WAIT_* in "
                   "quad-cycles, SQ_INSTS_* in wave-instructions; FETCH_SIZE doubled (gfx950 wide-read correction).",
           "timing_us": {"k_density_pair": us_pair, "k_density_plan": us_plan}}
    for k in ("k_density_pair", "k_density_plan"):
        out[k] = dict(d1.get(k, {}))
        out[k].update(d2.get(k, {}))
        if k in dt:
            out[k].update({kk: dt[k][kk] for kk in ("fetch_bytes", "write_bytes", "hbm_bytes")})
    p = out["k_density_pair"]
    if "SQ_INSTS_VALU" in p and "SQ_ACTIVE_INST_ANY" in p:
        p["derived"] = {
            "valu_ginst_s": round(p["SQ_INSTS_VALU"] / us_pair / 1e3, 1),
            "valu_frac_of_1228.8": round(p["SQ_INSTS_VALU"] / us_pair / 1e3 / 1228.8, 3),
            "wave_life_cycles": round(p["SQ_WAVE_CYCLES"] * 4 / p["SQ_WAVES"]),
            "active_frac": round(p["SQ_ACTIVE_INST_ANY"] / p["SQ_WAVE_CYCLES"], 3),
            "wait_any_frac": round(p["SQ_WAIT_ANY"] / p["SQ_WAVE_CYCLES"], 3),
            "wait_inst_frac": round(p["SQ_WAIT_INST_ANY"] / p["SQ_WAVE_CYCLES"], 3)}
    if "--lib" in sys.argv:
        lib = sys.argv[sys.argv.index("--lib") + 1]
        out["_build"] = {"lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(), "lib": lib}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(p.get("derived", {})))


if __name__ == "__main__":
    main()
