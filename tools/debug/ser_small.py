import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from dxa.ops import native, serialize as S
from dxa.engine.column import Table, column_from_pylist, PrimColumn
native.lib()
dev = torch.device("cuda", 0)
t = Table(["deviceId", "deviceType", "c"], [column_from_pylist([None, 5, None], "long", dev),
          column_from_pylist([None, "x", "y"], "string", dev), PrimColumn("long", torch.tensor([3, 4, 5], device=dev))])
st = S.Staged(t)
print("gpu", st.gpu)
print(list(st.render()))
