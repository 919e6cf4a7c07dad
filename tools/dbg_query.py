import sys, json, torch
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
import test_gpu_kernels as T
from dxa.engine.column import Table
from dxa.engine.expr import EvalContext
from dxa.engine.query import Catalog, run_sql
from dxa.engine.serialize import table_to_json_lines
gpu = torch.device("cuda:0")
cpu_raw, _, gpu_raw, _ = T._parse_both(gpu, n=5000, seed=3)
res = []
for raw in (cpu_raw, gpu_raw):
    cat = Catalog(); ctx = EvalContext(now_us=1551394800_000000); base = Catalog()
    base.register("T", Table(["Raw"], [raw]))
    cat.register("D", run_sql("SELECT Raw.*, current_timestamp() AS eventTimeStamp FROM T", base, ctx))
    q1 = run_sql("SELECT deviceDetails.deviceId, deviceDetails.deviceType, deviceDetails.homeId, COUNT(*) AS c FROM D "
                 "GROUP BY deviceId, deviceType, homeId ORDER BY deviceId, deviceType, homeId", cat, ctx)
    q1b = run_sql("SELECT deviceDetails.deviceId, deviceDetails.deviceType, deviceDetails.homeId, COUNT(*) AS c FROM D "
                 "GROUP BY deviceId, deviceType, homeId", cat, ctx)
    res.append((q1.to_pylist(), table_to_json_lines(q1), sorted(json.dumps(r, sort_keys=True) for r in q1b.to_pylist())))
print("groups", len(res[0][0]), len(res[1][0]))
print("unordered sets equal", res[0][2] == res[1][2])
print("ordered pylist equal", res[0][0] == res[1][0])
print("json equal", res[0][1] == res[1][1])
for i, (a, b) in enumerate(zip(res[0][0], res[1][0])):
    if a != b:
        print(i, a, b); break
for i, (a, b) in enumerate(zip(res[0][1], res[1][1])):
    if a != b:
        print(i, a, b); break
