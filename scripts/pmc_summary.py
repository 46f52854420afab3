"""Summarise rocprofv3 --pmc CSVs: per kernel, mean counter value per dispatch."""
import csv, glob, sys, collections
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/*counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        # a dispatch appears once per counter; values are summed over XCDs/SEs already
        print(f"   {c:28s} {sum(v)/len(v):16.1f}   (n={len(v)})")
