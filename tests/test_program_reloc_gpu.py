"""r06: step programs read each step's input row in place (csrc/program.hip
fh_program_relocate / fh_program_launch_at): the recorded launches' pointers into the per-step
slot are rewritten to row g of the round's rows, and the copy_bytes launch per step is gone.
A CIFAR10CNN round (ragged steps, dropout) and a SimpleCNN round (uint8 images, the gather
inside conv1) in program mode: every trained row bit-identical with the relocation on, with
it off (the copy into the slot) and in the eager round; the programs really relocated."""
import pytest
import torch

from fedhip import engine as eng_mod
from fedhip import ops
from fedhip.engine import PackedTrainer
from src.shared import models_pytorch as hm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _round(name, kw, sizes, mode, relocate, u8=False):
    prev = eng_mod.RELOCATE[0]
    eng_mod.RELOCATE[0] = relocate
    try:
        torch.manual_seed(0)
        model = hm.ModelFactory.create_model(name, **kw).to(DEV)
        eng = PackedTrainer(model, capacity=len(sizes), batch=32, device=DEV)
        if mode == "eager":
            eng.use_graphs = False
        else:
            eng.launch_mode = "program"
        for k in range(len(sizes)):
            eng.load_module_state(k, model)
        g = torch.Generator().manual_seed(5)
        shape = (1, 28, 28) if name == "simple_cnn" else (3, 32, 32)
        data = torch.randn(sum(sizes), *shape, generator=g).to(DEV)
        labels = torch.randint(0, 10, (sum(sizes),), generator=g).to(DEV)
        offs = [sum(sizes[:k]) for k in range(len(sizes))]
        gen = torch.Generator().manual_seed(11)
        for r in range(2):
            plan = eng.make_plan(sizes, 1, generator=gen)
            eng.run_round(data, labels, offs, plan, "sgd", 1e-2, seed=r)
        torch.cuda.synchronize()
        progs = [p for _, p in eng._graphs.values() if p is not None]
        relocs = [p.relocs for p in progs]
        return eng.params[:len(sizes)].clone(), eng.bufs[:len(sizes)].clone(), relocs
    finally:
        eng_mod.RELOCATE[0] = prev


@pytest.mark.parametrize("name,kw", [("cifar10_cnn", {"dropout_rate": 0.3}),
                                     ("simple_cnn", {})])
def test_relocated_programs_bit_identical(name, kw):
    sizes = [100, 70, 37, 9]
    p_e, b_e, _ = _round(name, kw, sizes, "eager", True)
    p_r, b_r, rel_on = _round(name, kw, sizes, "program", True)
    p_c, b_c, rel_off = _round(name, kw, sizes, "program", False)
    assert rel_on and all(r > 0 for r in rel_on), rel_on  # every program relocated
    assert all(r == 0 for r in rel_off)
    assert torch.equal(p_r, p_c) and torch.equal(b_r, b_c)
    assert torch.equal(p_r, p_e) and torch.equal(b_r, b_e)
