"""Per-kernel durations from a rocprofv3 kernel trace csv.  usage: trace_summ.py TRACE.csv [N]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    nm = re.sub(r'\(anonymous namespace\)::', '', r['Kernel_Name']).split('(')[0].split('::')[-1]
    d[nm].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
for k, v in sorted(d.items(), key=lambda x: -max(x[1]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    print('%-28s n=%-3d max %8.3f ms' % (k, len(v), max(v)))
