import torch, sys
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from pose_estimation_amd import ops, _lib
from pose_estimation_amd.runtime import P, ptr
import torch.nn as nn
dev = torch.device('cuda', 0)
B, HW, cout, co, oc, Cx = 1, 32, 72, 0, 0, 72
cin = 128
g = torch.Generator().manual_seed(1)
conv = nn.Conv2d(cin, cout, 1, bias=True)
with torch.no_grad():
    conv.weight.copy_(0.1 * torch.randn(conv.weight.shape, generator=g)); conv.bias.copy_(torch.randn(cout, generator=g))
x = torch.randn(B, cin, 1, HW, generator=g)
ref = conv(x).detach()
xa = ops.new_act(B, 1, HW, cin, dev); xa.t[...] = x.permute(0, 2, 3, 1).to(dev)
spec = ops.make_conv(conv.float(), None, dev, cin_p=cin)
w3 = ops.quad_weights_x3(spec.wt[0], ops.pad4(cout), cin)
out = torch.full((B, Cx, 1, HW), float('nan'), device=dev)
_lib.check(_lib.lib().krrn_conv1x1_nchw_x3_f32(ptr(xa.t), xa.cs, xa.co, B, HW, cin, ptr(w3), ops.pad4(cout), cout, ptr(spec.scale), ptr(spec.bias), ptr(out), Cx, oc, P(torch.cuda.current_stream().cuda_stream)), "x3")
torch.cuda.synchronize()
got = out.cpu()
print("nan", int(torch.isnan(got).sum()), "zero", int((got == 0).sum()), "of", got.numel())
for n in range(0, 20):
    print(n, [round(float(v), 3) for v in got[0, n, 0, :6]], [round(float(v), 3) for v in ref[0, n, 0, :6]])
# is any got value equal to a ref value elsewhere?
rf = ref.flatten()
for n, p in [(0, 0), (1, 0), (4, 0), (16, 0), (17, 3)]:
    v = got[0, n, 0, p]
    idx = (torch.abs(rf - v) < 1e-4).nonzero().flatten().tolist()
    print("got", n, p, float(v), "matches ref at", [(i // HW, i % HW) for i in idx[:4]])
