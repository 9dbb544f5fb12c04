"""Probe: the training step's spatial-weights MLP (16x256, F=128) backward on the HIP slab kernel
(nrt_mlp_backward) against a layer-by-layer formulation on library GEMMs (torch.matmul ->
rocBLAS / hipBLASLt, FP32 with TF32-like modes off), same rows; timing only."""
import sys
import time

import torch

sys.path.insert(0, ".")


def main():
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    torch.backends.cuda.matmul.allow_tf32 = False
    set_precision("fp32")
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for M, (L, H, F, out) in ((19200, (16, 256, 128, 8)), (19200, (10, 256, 16, 3)),
                              (19200, (6, 96, 64, 3))):
        mlp = SkipConnMLP(num_layers=L, hidden_size=H, in_size=3, out=out, freqs=F,
                          device="cpu").to(dev)
        x = torch.rand(M, 3, device=dev) - 0.5
        dy = torch.randn(M, out, device=dev)

        def hip():
            xm = x.clone().requires_grad_(True)
            (mlp(xm) * dy).sum().backward()

        # the reference's eager SkipConnMLP (neural_blocks.py:75-86) under torch autograd
        def eager():
            xm = x.clone().requires_grad_(True)
            enc = torch.cat([xm, torch.sin(xm @ mlp.basis_p), torch.cos(xm @ mlp.basis_p)], -1)
            act = torch.nn.functional.leaky_relu
            h = mlp.init(enc)
            for i, lay in enumerate(mlp.layers):
                if i != L - 1 and i % 3 == 0:
                    h = torch.cat([h, enc], -1)
                h = lay(act(h))
            y = mlp.out(act(h))
            (y * dy).sum().backward()

        for name, f in (("hip", hip), ("eager_gemm", eager)):
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                f()
            torch.cuda.synchronize()
            print(f"L{L} H{H} F{F} M{M} {name}: {(time.perf_counter() - t0) / 10 * 1e3:.2f} ms "
                  "(forward + backward)", flush=True)


if __name__ == "__main__":
    main()
