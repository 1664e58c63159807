import sqlite3, collections, sys
c = sqlite3.connect(sys.argv[1])
names = {kid: n for kid, n in c.execute("select id, kernel_name from kernel_symbols")} if False else {}
rows = c.execute("select dispatch_id, kernel_id, counter_name, value, duration, grid_size_y from counters_collection order by dispatch_id")
per = collections.OrderedDict()
for d, kid, cn, v, dur, gy in rows:
    e = per.setdefault(d, {"kid": kid, "dur": dur, "gy": gy, "c": collections.defaultdict(float)})
    e["c"][cn] += v
sym = {}
for r in c.execute("select * from kernel_symbols limit 1"):
    pass
cols = [x[0] for x in c.execute("select * from kernel_symbols limit 1").description]
for r in c.execute("select * from kernel_symbols"):
    d = dict(zip(cols, r)); sym[d.get("id") or d.get("kernel_id")] = d.get("kernel_name") or d.get("formatted_kernel_name") or d.get("name")
disp = list(per.items())
print(len(disp), "dispatches")
# order: stamp-all(1MiB), then 20x (stamp, verify) at 1 MiB; stamp-all(2MiB), 20x (stamp, verify) at 2 MiB (+ verify after stamp-all)
groups = collections.defaultdict(list)
half = len(disp) // 2
for i, (d, e) in enumerate(disp):
    stride = "1MiB" if i < half else "2MiB"
    k = ("verify" if "verify" in (sym.get(e["kid"]) or "") else "stamp")
    groups[(stride, k)].append(e)
keys = ["duration", "SQ_WAVES", "TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_DRAM_sum", "TCC_HIT_sum", "TCC_MISS_sum", "TCP_UTCL1_REQUEST_sum", "TCP_UTCL1_TRANSLATION_HIT_sum", "TCP_UTCL1_TRANSLATION_MISS_sum", "TCP_UTCL1_STALL_MULTI_MISS_sum"]
print("| stride | kernel | n | " + " | ".join(keys) + " |")
print("|---|---|---:|" + "---:|" * len(keys))
for (stride, k), es in sorted(groups.items()):
    es = es[1:]  # skip the first (stamp-all / its verify)
    avg = lambda f: sum(f(e) for e in es) / len(es)
    vals = [avg(lambda e: (e["dur"] or 0) / 1e3)] + [avg(lambda e, kk=kk: e["c"].get(kk, 0)) for kk in keys[1:]]
    print(f"| {stride} | {k} | {len(es)} | " + " | ".join(f"{v:,.1f}" for v in vals) + " |")
