"""print the orbgpu kernels of a rocprofv3 kernel_stats.csv: name, calls, average ms"""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    if "orbgpu" in r["Name"]:
        name = r["Name"].replace("void ", "").replace("orbgpu::(anonymous namespace)::", "").split("(")[0]
        print(f"{name[:48]:48s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e6:8.4f} ms")
