"""Step-by-step replay of test_mlp_backward_refuses_weights_changed_after_forward with a device
synchronisation and a flushed print after every library call (debug aid)."""
import sys
import torch
sys.path.insert(0, ".")
from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
from neural_raytracing_amd.pathtracer._handles import train_handle
from neural_raytracing_amd import _lib


def say(*a):
    print(*a, flush=True)


torch.manual_seed(3)
m = SkipConnMLP(num_layers=2, hidden_size=32, out=2, device="cuda").cuda()
x = torch.rand(64, 3, device="cuda")
say("pack"); h = train_handle(m); torch.cuda.synchronize(); say("packed")
y = m(x).square().sum(); torch.cuda.synchronize(); say("forward 1 ok")
with torch.no_grad():
    m.out.weight.add_(1.0)
say("refresh"); h2 = train_handle(m); torch.cuda.synchronize(); say("refreshed", h2 is h)
y2 = m(x).square().sum(); torch.cuda.synchronize(); say("forward 2 ok")
mode = sys.argv[1] if len(sys.argv) > 1 else "thread"
if mode == "main":
    # call the backward entry point from the main thread
    g = torch.autograd.grad(y2, list(m.parameters()))
else:
    y2.backward()
torch.cuda.synchronize(); say("backward ok")
