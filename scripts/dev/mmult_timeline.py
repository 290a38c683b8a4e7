"""One replay round's kernel timeline and the dispatches per round, from a rocprofv3
--kernel-trace CSV of `bench.py --workload mmult` (two replays of 250 rounds each).
Usage: python scripts/dev/mmult_timeline.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
tw = [i for i, r in enumerate(rows) if "twin_kernel" in r["Kernel_Name"]]
rounds = len(tw)
per = collections.Counter(r["Kernel_Name"].split("(")[0][:60] for r in rows[tw[0]:])
print(f"rounds traced: {rounds}; dispatches per round (from the first twin on):")
for k, v in per.most_common():
    print(f"  {v / rounds:5.2f}  {k}")
s = tw[-100] - 4
t0 = int(rows[s]["Start_Timestamp"])
print("one round (us from the first line; queue, start, end, duration, kernel):")
for r in rows[s:tw[-99] + 1]:
    st = (int(r["Start_Timestamp"]) - t0) / 1000
    en = (int(r["End_Timestamp"]) - t0) / 1000
    print(f"  q{r['Queue_Id']} {st:8.2f} {en:8.2f} {en - st:6.2f}  {r['Kernel_Name'][:60]}")
a, b = int(rows[tw[-200]]["Start_Timestamp"]), int(rows[tw[-1]]["Start_Timestamp"])
print(f"round period under the tracer (last 200 rounds): {(b - a) / 199 / 1000:.1f} us")
