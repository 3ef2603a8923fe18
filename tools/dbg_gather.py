import ctypes, sys, os
sys.path.insert(0, os.getcwd())
import torch, fluere_amd
from fluere_amd import _lib
L = _lib.lib()
cfg = fluere_amd.synth_cfg(_lib.SYNTH_IMIX, 160_000, 4000, 0xF10E0004)
G, per, cap = 4, 40000, 1024
blk = int(L.fluere_shard_block_bytes(cap))
buf = torch.zeros(G * blk, dtype=torch.uint8, device="cuda")
ctxs = []
for r in range(G):
    ctx = fluere_amd.FlowContext(max_flows=1 << 16)
    b, o, nbytes = fluere_amd.synth_device(cfg, r * per, per)
    L.fluere_set_index_base(ctx._h, r * per)
    ctx.add_device_batch(b, nbytes, o, per)
    torch.cuda.synchronize()
    ctx.parse_aggregate()
    print("export rc", L.fluere_export_device(ctx._h, buf.data_ptr() + r * blk, cap))
    ctxs.append(ctx)
torch.cuda.synchronize()
print("hdrs", buf.view(G, blk)[:, :64].contiguous().view(torch.int64).cpu().tolist())
m = fluere_amd.FlowContext(max_flows=1 << 16)
st = _lib.Stats()
rc = L.fluere_merge_gathered(m._h, buf.data_ptr(), G, cap, ctypes.byref(st))
print("rc", rc, st.as_dict())
