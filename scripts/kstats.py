"""Print a rocprofv3 kernel_stats.csv compactly: average microseconds, calls, name."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("mochi::", "")
    print(f'{float(r["AverageNs"]) / 1e3:10.1f} us  x{r["Calls"]:>4}  {n[:70]}')
