"""Absolute VALU issue costs on gfx950 from a rocprofv3 PMC run of scripts/ubench_issue:
  rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d <dir> -o run -- scripts/ubench_issue
  python scripts/issue_costs.py <dir> <tag>   -> profiles/<tag>_issue_costs.json
Per kernel (one instruction repeated by 8 waves per SIMD in 8 independent chains), the cost is the
dispatch's SIMD-cycles, 1024 x GRBM_GUI_ACTIVE / 8 (GRBM_GUI_ACTIVE summed over the 8 XCDs), over
its VALU wave-instructions: SIMD-cycles per wave64 instruction at full occupancy, including the
kernel's ramp and its few non-loop instructions (< 1 % of the count)."""
import collections
import csv
import glob
import json
import os
import sys

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
f = glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True)[0]
per = collections.defaultdict(lambda: collections.defaultdict(dict))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
    per[k][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
name = {"k_fma_f64": "v_fma_f64", "k_add_f64": "v_add_f64", "k_mul_f64": "v_mul_f64", "k_fma_f32": "v_fma_f32",
        "k_add_u32": "v_add_u32", "k_bitop3": "v_bitop3_b32", "k_alignbit": "v_alignbit_b32",
        "k_mul_lo_u32": "v_mul_lo_u32", "k_mul_hi_u32": "v_mul_hi_u32", "k_mad_u64_u32": "v_mad_u64_u32",
        "k_lshl_b64": "v_lshlrev_b64", "k_cvt_f64_u32": "v_cvt_f64_u32", "k_cvt_f64_i32": "v_cvt_f64_i32",
        "k_rsq_f64": "v_rsq_f64", "k_rcp_f64": "v_rcp_f64", "k_ldexp_f64": "v_ldexp_f64", "k_max_f64": "v_max_f64",
        "k_fract_f64": "v_fract_f64", "k_cndmask": "v_cndmask_b32", "k_med3_i32": "v_med3_i32",
        "k_pk_fma_f32": "v_pk_fma_f32", "k_mul_u32_u24": "v_mul_u32_u24", "k_pk_sub_u16": "v_pk_sub_u16",
        "k_pk_min_u16": "v_pk_min_u16", "k_bcnt": "v_bcnt_u32_b32", "k_cvt_f32_f64": "v_cvt_f32_f64",
        "k_cvt_pknorm": "v_cvt_pknorm_u16_f32", "k_min_f64": "v_min_f64"}
costs, clocks = {}, {}
for k, ds in per.items():
    if k not in name:
        continue
    last = ds[max(ds)]          # the second (warm) dispatch
    costs[name[k]] = round(1024 * last["GRBM_GUI_ACTIVE"] / 8 / last["SQ_INSTS_VALU"], 3)
out = {"calibration": "absolute", "waves_per_simd": 8,
       "method": "rocprofv3 PMC: 1024 x GRBM_GUI_ACTIVE / 8 over SQ_INSTS_VALU per dispatch (scripts/issue_costs.py)",
       "cycles_per_wave_instruction": dict(sorted(costs.items()))}
p = os.path.join(root, "profiles", f"{tag}_issue_costs.json")
json.dump(out, open(p, "w"), indent=1)
print(json.dumps(out))
