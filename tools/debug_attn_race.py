import sys; sys.path.insert(0, '/root/repo/sam-quantization_amd')
import torch
from samq import ops
torch.manual_seed(0)
dev = torch.device('cuda')
hw, heads, d = 64, 16, 80
c = heads * d
q1 = (torch.randn(1, hw, hw, 3 * c, device=dev) * 0.5).half()
rh = (torch.randn(2 * hw - 1, d, device=dev) * 0.1).half()
rw = (torch.randn(2 * hw - 1, d, device=dev) * 0.1).half()
outs = [ops.rel_attention(q1, None, rh, rw, heads, 0, d ** -0.5) for _ in range(6)]
base = outs[0].float()
for i, o in enumerate(outs[1:]):
    dd = (o.float() - base).abs().view(hw, hw, heads, d)
    nz = dd > 0
    print(f"run {i+1}: differing elems {int(nz.sum())}, max {dd.max().item():.2e}")
    if nz.any():
        idx = nz.nonzero()
        print("  rows", sorted(set(idx[:, 0].tolist()))[:20], "cols mod16", sorted(set((idx[:, 1] % 16).tolist()))[:16])
        print("  heads", sorted(set(idx[:, 2].tolist())), "d", sorted(set(idx[:, 3].tolist()))[:20])
        tiles = sorted(set((idx[:, 0] * 4 + idx[:, 1] // 16).tolist()))
        print("  q-tiles", tiles[:30], "qblock(16 tiles)", sorted(set(t // 16 for t in tiles)))
