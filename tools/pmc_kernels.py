"""Dev tool: average PMC counter values per kernel (by name) from rocprofv3
--pmc passes over tools/pmc_traffic.py's in-step workload.

  rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES ... --output-format csv -d DIR -o run -- python tools/pmc_traffic.py run
  python tools/pmc_kernels.py DIR [name-filter ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name[:name.index("(")].replace("void ", "") if "(" in name else name


def main(d, *filt):
    vals = defaultdict(lambda: defaultdict(list))
    grid = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"]) + f" g{r['Grid_Size']}"
            if filt and not any(x in k for x in filt):
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            grid[k] = r
    for k in sorted(vals):
        cs = vals[k]
        r = grid[k]
        print(f"{k}  vgpr {r['VGPR_Count']} agpr {r['Accum_VGPR_Count']} lds {r['LDS_Block_Size']} wg {r['Workgroup_Size']}")
        print("   " + "  ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items())))


if __name__ == "__main__":
    main(*sys.argv[1:])
