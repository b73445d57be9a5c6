import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
orders = sys.argv[2].split(",")
seq = [r for r in rows if "classify_kernel" in r["Kernel_Name"]]
per = 26  # 13 classify calls x 2 launches per ordering
for i, o in enumerate(orders):
    chunk = seq[i * per:(i + 1) * per][6:]  # drop warmup
    d = collections.defaultdict(list)
    for r in chunk:
        stage = r["Kernel_Name"].split("<")[1].split(",")[2].strip()
        d[stage].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    print(o, {k: round(sum(v) / len(v), 3) for k, v in d.items()})
