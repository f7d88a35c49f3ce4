# Summarise a rocprofv3 counter_collection.csv per kernel (sums over dispatches).
import csv, glob, collections, sys
f = glob.glob(sys.argv[1] + '/*counter_collection.csv')[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'].replace('(anonymous namespace)', 'anon').split('(')[0].split('::')[-1]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in acc.items():
    print(k, ' '.join(f"{a}={b:.3g}" for a, b in sorted(v.items())))
