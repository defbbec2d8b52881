import csv, sys
from collections import Counter, defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "k_sumsq" in r["Kernel_Name"]]
step = rows[adam[-2] + 1:adam[-1] + 1]
c=defaultdict(float); n=Counter()
for r in step:
    k=(r['Queue_Id'], r['Stream_Id']); c[k]+= (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6; n[k]+=1
for k in sorted(c): print(k, n[k], round(c[k],2))
