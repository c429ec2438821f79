"""bench.py's rigid microbench (the settled pile fixture) and the C1/C3 tick rates for A/B runs:
LPE_LIB=... python profiles/rigid_ab.py"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
lpe = bench._load("lpe", os.path.join(bench.PKG, "lpe.py"))
r = bench.rigid_microbench(lpe, 0)
print(json.dumps({"lib": os.environ.get("LPE_LIB", "default"), "step_us": r["step_kernels_us"],
                  "pgs": r["kernels_us"].get("k_pgs_stripes"), "pos": r["kernels_us"].get("k_pos_stripes"),
                  "colours": r["colours"]}), flush=True)
