import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "rust-crdt_amd")
import crdts_hip, map_slab
import map_kat_runner as mkr
from test_gpu_map_nested import gpu_merge
eng = crdts_hip.Engine(0)
case = [c for c in mkr.load_cases(nested=True) if c["name"] == "test_merge_deferred_remove"][0]
class B(mkr.PyMapBackend):
    def merge(self, dst, src):
        exp = dst.clone(); exp.merge(src)
        out = gpu_merge(eng, dst, src)
        print("MERGE dst", dst.canonical()); print("  src", src.canonical()); print("  exp", exp.canonical()); print("  got", out.canonical())
        dst.clock, dst.entries, dst.deferred = out.clock, out.entries, out.deferred
try:
    mkr.run_case(case, B())
except AssertionError as e:
    print("ASSERT", e)
import torch, numpy as np
sc = eng._map_map_scratch
print("tsrc", sc[:128].cpu().numpy().view(np.uint64)[:16])
# direct: a 1-object nested merge of m2-like state with an empty map
m2 = mkr.nested_map()
mkr.apply_raw(m2, {"up": {"dot": [0, 1], "key": 1, "op": {"up": {"dot": [0, 1], "key": 1, "op": {"put": {"clock": [[0, 1]], "val": 7}}}}}})
from test_gpu_map_nested import INNER, CAPS
S = crdts_hip.MapMapSlab.alloc(1, 1, inner_caps=INNER, **CAPS)
O = crdts_hip.MapMapSlab.alloc(1, 1, inner_caps=INNER, **CAPS)
map_slab.nested_map_to_row(m2, O, 0, 1)
print("O inner n_keys", O.inner.a["n_keys"][:4], "O n_keys", O.a["n_keys"])
R = eng.map_map_merge(S.to("cuda"), O.to("cuda"), 1)
torch.cuda.synchronize()
print("tsrc", sc[:128].cpu().numpy().view(np.uint64)[:16])
H = R.host()
print("R n_keys", H.a["n_keys"], "inner n_keys", H.inner.a["n_keys"], "inner clock", H.inner.a["clock"][:4].ravel())
raw = sc[:512].cpu().numpy()
print("Tb", raw[128:192].view(np.uint64))
print("Tmp clock", raw[192:256].view(np.uint64), "Tmp n_keys", raw[256:288].view(np.uint32))
print("status", eng.status() if hasattr(eng, "status") else None)
