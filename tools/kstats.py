import csv, collections, statistics, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r['Kernel_Name'].split('(')[0]
    if any(x in n for x in sys.argv[2].split(',')):
        d[(n[:50], r['Grid_Size_X'], r['Grid_Size_Y'])].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000)
for k, v in sorted(d.items()):
    print(k, len(v), 'median', round(statistics.median(v),2), 'min', round(min(v),2), 'max', round(max(v),2))
