"""fp64 floating-point work per kernel launch from one rocprofv3 --pmc pass
(SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64, SQ_INSTS_VALU_MFMA_MOPS_F64, SQ_WAVES):
flops = 64 (ADD + MUL + TRANS) + 128 FMA + 512 MFMA_MOPS (the MOPS counter is
add/mul operations / 512). Wave-instruction counts are scaled by all 64 lanes,
so lanes masked off (partial segments) are counted too: an upper bound of the
arithmetic the kernel issues. Writes a JSON summary that bench.py reports next
to the HBM roofline ("report max(bytes/BW_peak, flops/FP64_peak)
and name the binding one").

    python tools/pmc_flops.py run_counter_collection.csv out.json [config]
"""
import collections
import csv
import json
import statistics
import sys


def main():
    path, out = sys.argv[1:3]
    config = sys.argv[3] if len(sys.argv) > 3 else "c2"
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kernels = {}
    for name, c in per.items():
        med = {k: statistics.median(v) for k, v in c.items()}
        valu = 64.0 * (med.get("SQ_INSTS_VALU_ADD_F64", 0.0) + med.get("SQ_INSTS_VALU_MUL_F64", 0.0)
                       + med.get("SQ_INSTS_VALU_TRANS_F64", 0.0)) + 128.0 * med.get("SQ_INSTS_VALU_FMA_F64", 0.0)
        mfma = 512.0 * med.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0)
        if valu + mfma == 0.0:
            continue
        kernels[name] = {"dispatches": len(c.get("SQ_WAVES", [])), "waves": med.get("SQ_WAVES", 0.0),
                         "fp64_valu_flops": valu, "fp64_mfma_flops": mfma, "fp64_flops": valu + mfma}
    json.dump({"config": config, "kernels": kernels,
               "method": "rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 "
                         "SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES (one pass), median over "
                         "dispatches; flops = 64 (ADD+MUL+TRANS) + 128 FMA + 512 MFMA_MOPS per wave-instruction "
                         "count (all 64 lanes counted)"},
              open(out, "w"), indent=1)
    for k, v in kernels.items():
        print(f"{k[:48]:48s} {v['fp64_flops'] / 1e9:8.3f} GFLOP (MFMA {v['fp64_mfma_flops'] / 1e9:.3f})")


if __name__ == "__main__":
    main()
