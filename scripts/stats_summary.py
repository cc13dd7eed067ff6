"""Short table of a rocprofv3 kernel_stats.csv: kernel (template args kept), calls, total ms, avg us, %."""
import csv, re, sys
for path in sys.argv[1:]:
    print(path)
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(.*", "", r["Name"]).replace("void ", "")
        print(f"  {name[:48]:48s} calls={int(r['Calls']):5d} total={float(r['TotalDurationNs'])/1e6:9.3f} ms "
              f"avg={float(r['AverageNs'])/1e3:9.2f} us  {float(r['Percentage']):6.2f}%")
