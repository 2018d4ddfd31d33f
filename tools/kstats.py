"""Print a rocprofv3 kernel_stats.csv as name / calls / avg ms / share."""
import csv
import sys

for path in sys.argv[1:]:
    print("==", path)
    for x in csv.DictReader(open(path)):
        print(f"{x['Name'][:70]:70s} {x['Calls']:>5s} avg_ms={float(x['AverageNs'])/1e6:9.4f} pct={float(x['Percentage']):6.2f}")
