import sys; sys.path.insert(0, '/root/repo/sam-quantization_amd')
import torch
from samq import ops
torch.manual_seed(0)
dev = torch.device('cuda')
for (hw, win, heads, d) in ((64, 0, 16, 80), (64, 14, 16, 80), (64, 0, 12, 64), (32, 0, 4, 80)):
    c = heads * d
    q1 = (torch.randn(1, hw, hw, 3 * c, device=dev) * 0.5).half()
    q2 = torch.cat([q1, (torch.randn(1, hw, hw, 3 * c, device=dev) * 0.5).half()])
    side = win or hw
    rh = (torch.randn(2 * side - 1, d, device=dev) * 0.1).half()
    rw = (torch.randn(2 * side - 1, d, device=dev) * 0.1).half()
    b = (torch.randn(3 * c, device=dev) * 0.1).half()
    o1 = ops.rel_attention(q1, b, rh, rw, heads, win, d ** -0.5)
    o2 = ops.rel_attention(q2, b, rh, rw, heads, win, d ** -0.5)
    o1b = ops.rel_attention(q1, b, rh, rw, heads, win, d ** -0.5)
    print(hw, win, heads, d, "batch diff", (o1 - o2[:1]).abs().max().item(), "rerun diff", (o1 - o1b).abs().max().item())
