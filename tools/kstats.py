"""Print a rocprofv3 *_kernel_stats.csv as an aligned table (names contain commas)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:10.1f} pct={float(r['Percentage']):6.2f}")
