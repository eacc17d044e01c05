"""Resume (new; the reference only saves its generator, capgan.py:185-200): a run of two
workers over gloo interrupted after 2 rounds and resumed from the per-worker resume files (a NEW
Driver, as a restarted process would build it) ends bitwise where the uninterrupted 4-round run ends --
G, G running statistics, D, and lambda -- on the CPU stand-in step (tests/dist_oracle_step.py).
Cases: CAPGAN with the E-share every round, and MD-GAN with the D-swap every round (the swap
permutations come from the server's Random(server + 100), whose state travels in the resume file).
Ranks whose resume files hold different rounds refuse to start, and a file that fails to load on one
rank makes every rank raise (no rank left waiting in a collective)."""
import os
import tempfile

import pytest

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_driver_gloo import _cfg, _free_port

KW = dict(algo="capgan", num_workers=2, num_servers=1, share_every=1)
KW_SWAP = dict(algo="mdgan", num_workers=2, num_servers=1, swap_every=1)


def _proc(rank, world, port, outdir, mode, kw=KW):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cglgan.driver import Driver
        from dist_oracle_step import oracle_step_factory
        if mode == "straight":
            drv = Driver(_cfg(**kw), step_factory=oracle_step_factory, device="cpu")
            drv.run(4, log=None)
        else:
            rd = os.path.join(outdir, "resume")
            first = Driver(_cfg(resume_dir=rd, **kw), step_factory=oracle_step_factory, device="cpu")
            assert first.round == 0
            first.run(2, log=None)                      # writes resume-<algo>-rank{r}.pt at the end
            del first
            if mode == "torn" and rank == 1:            # a crash before rank 1 replaced its file
                os.remove(os.path.join(rd, f"resume-{kw['algo']}-rank1.pt"))
            if mode == "corrupt" and rank == 1:         # a damaged file: only rank 1's load raises
                with open(os.path.join(rd, f"resume-{kw['algo']}-rank1.pt"), "wb") as f:
                    f.write(b"not a checkpoint")
            dist.barrier()
            if mode == "corrupt":
                # every rank must raise (rank 0 too, from the shared all-reduce) instead of rank 0 waiting
                # in a collective for the process-group timeout
                try:
                    Driver(_cfg(resume_dir=rd, **kw), step_factory=oracle_step_factory, device="cpu")
                    msg = "no error"
                except Exception as e:
                    msg = f"{type(e).__name__}: {e}"
                with open(os.path.join(outdir, f"corrupt{rank}.txt"), "w") as f:
                    f.write(msg)
                return
            drv = Driver(_cfg(resume_dir=rd, **kw), step_factory=oracle_step_factory, device="cpu")
            assert drv.round == 2 and drv.step.round == 2
            drv.run(2, log=None)
        s = drv.step
        torch.save({"g": s.g_params, "r": s.g_running, "d": s.d_params, "lam": s.lsgd.lam.detach(),
                    "round": drv.round}, os.path.join(outdir, f"{mode}{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kw", [KW, KW_SWAP], ids=["capgan-eshare", "mdgan-dswap"])
def test_resume_bitwise_world2(kw):
    with tempfile.TemporaryDirectory() as td:
        for mode in ("straight", "resumed"):
            mp.spawn(_proc, args=(2, _free_port(), td, mode, kw), nprocs=2, join=True)
        for r in range(2):
            a = torch.load(os.path.join(td, f"straight{r}.pt"), weights_only=True)
            b = torch.load(os.path.join(td, f"resumed{r}.pt"), weights_only=True)
            assert a["round"] == b["round"] == 4
            for k in ("g", "r", "d", "lam"):
                assert torch.equal(a[k], b[k]), (r, k)
        assert os.path.exists(os.path.join(td, "resume", f"resume-{kw['algo']}-rank1.pt"))


def test_dswap_resume_changes_nothing_but_the_generator():
    """Without the saved generator state the resumed MD-GAN run would restart the permutation sequence:
    the 4 permutations of an uninterrupted run differ from 2 + 2 restarted ones (so the case above
    really exercises the saved state)."""
    from cglgan.exchange import DSwap
    a = DSwap(2, 0)
    straight = [a.next_perm() for _ in range(4)]
    b, c = DSwap(2, 0), DSwap(2, 0)
    restarted = [b.next_perm() for _ in range(2)] + [c.next_perm() for _ in range(2)]
    assert straight != restarted


def test_resume_rounds_must_agree_world2():
    with tempfile.TemporaryDirectory() as td:
        with pytest.raises(Exception, match="different rounds"):
            mp.spawn(_proc, args=(2, _free_port(), td, "torn", KW), nprocs=2, join=True)


def test_resume_load_failure_raises_on_every_rank():
    """a resume file that fails to load on one rank makes every rank raise together."""
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_proc, args=(2, _free_port(), td, "corrupt", KW), nprocs=2, join=True)
        m0 = open(os.path.join(td, "corrupt0.txt")).read()
        m1 = open(os.path.join(td, "corrupt1.txt")).read()
        assert "another rank failed to load" in m0, m0
        assert m1 != "no error" and "another rank" not in m1, m1


def test_resume_file_roundtrip(tmp_path):
    from cglgan.checkpoint import load_resume, save_resume

    class S:
        def __init__(self):
            self.x = torch.arange(4.0)

        def resume_state(self):
            return {"x": self.x.clone()}

        def load_resume_state(self, sd):
            self.x.copy_(sd["x"])

    a, b = S(), S()
    b.x.zero_()
    p = save_resume(a, str(tmp_path / "r.pt"), round=7, config="k")
    meta = load_resume(b, p)
    assert meta == {"round": 7, "config": "k"} and torch.equal(b.x, a.x)
