"""Summarise a rocprofv3 kernel trace: per (kernel, grid) average durations."""
import collections
import csv
import sys


def main(path, top=40):
    rows = list(csv.DictReader(open(path)))
    d = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        short = name.split("(")[0] if not name.startswith("(") else name.split("(")[1].split(")")[-1]
        short = name[:70]
        d[(short, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])].append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in d.values())
    print(f"total {tot / 1e6:.3f} ms over {len(rows)} launches")
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print(f"{sum(v) / 1e6:8.3f}ms {len(v):5d} x {sum(v) / len(v) / 1e3:7.1f}us  grid={k[1]}x{k[2]}x{k[3]}  {k[0]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
