"""Per-kernel table of PMC counters from rocprofv3 --pmc passes (gpurun_out/pmcc/<pass>/...).
python scripts/pmc_table.py gpurun_out/pmcc"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        key = (r["Kernel_Name"].replace("void mgmc::", "")[:44], r["Grid_Size"])
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
cols = ["VALUBusy", "SALUBusy", "SQ_INSTS_VALU", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS", "FETCH_SIZE", "WRITE_SIZE",
        "GRBM_GUI_ACTIVE"]
print(f"{'kernel':44s} {'grid':>9s} " + " ".join(f"{c[:12]:>12s}" for c in cols))
rows = sorted(vals.items(), key=lambda kv: -sum(kv[1].get("GRBM_GUI_ACTIVE", [0])) / max(1, len(kv[1].get("GRBM_GUI_ACTIVE", [1]))))
for (name, grid), d in rows[:20]:
    print(f"{name:44s} {grid:>9s} " + " ".join(f"{(sum(d[c]) / len(d[c])) if d.get(c) else float('nan'):12.4g}" for c in cols))
