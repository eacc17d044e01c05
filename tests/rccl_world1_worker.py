"""Worker of tests/test_gpu_rccl_world1.py (run under torch.distributed.run, one process): the MLP and conv
exchange rounds over a ONE-rank RCCL group with the N > 1 code path forced (phase A, loss all-gather, alpha,
gradient all-reduce, phase B, E-share on the side stream), compared bitwise with the same rounds run
without a group.  Prints one line "RCCL-WORLD1 OK ..." on success."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cgl-gan_amd"), ROOT]


def mlp_step(B=64):
    from cglgan import GanStep, specs
    from cglgan.init import default_init
    gm, dm = specs.mnist_generator(), specs.mnist_discriminator()
    g = torch.Generator().manual_seed(5)
    real = (torch.rand(8 * B, 784, generator=g) * 2 - 1).cuda()
    st = GanStep(gm, dm, batch=B, loss="ce", weighting="capgan", n_workers=1, rank=0, gen_z=True, real=real,
                 sample_n=real.shape[0], seed=77)
    torch.manual_seed(20211212)
    default_init(gm, st.g_views)
    torch.manual_seed(555)
    default_init(dm, st.d_views)
    st.reset()
    return st


def main():
    from cglgan.exchange import DistComm, WorkerExchange
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
    assert dist.get_world_size() == 1 and dist.get_backend() == "nccl"
    a, b = mlp_step(), mlp_step()
    ex = WorkerExchange(a, DistComm(), share_every=1, force_split=True)
    ref = WorkerExchange(b, None)
    for r in range(4):
        ex.round(r, graph=(r % 2 == 1))
        ref.round(r, graph=(r % 2 == 1))
    torch.cuda.synchronize()
    for name in ("g_params", "g_m", "g_v", "d_params", "d_m", "d_v", "g_running"):
        x, y = getattr(a, name), getattr(b, name)
        assert torch.equal(x, y), (name, (x - y).abs().max().item())
    sa, sb = a.stats(), b.stats()
    assert sa["round"] == sb["round"] == 4 and sa["g_loss"] == sb["g_loss"] and sa["alpha"] == 1.0, (sa, sb)
    dist.destroy_process_group()
    print(f"RCCL-WORLD1 OK rounds=4 g_loss={sa['g_loss']:.6f} lambda={sa['lambda']:.6f}", flush=True)


if __name__ == "__main__":
    main()
