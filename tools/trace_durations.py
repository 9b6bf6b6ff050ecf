"""Per-launch kernel durations (us) in launch order from a rocprofv3 --kernel-trace csv."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 60
for r in rows[-last:]:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    name = name.split("(")[0]
    print(f"{name[:34]:<34} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000:9.1f}")
