"""Print per-parameter |hip-fp64| / tol for the ResNet Adam golden case."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import conftest  # noqa: F401  (paths)
import test_train_gpu as T

orig = T.check_params


def check(gpu_named, ref32, ref64, init, steps, lr, opt):
    p64s = dict(ref64.named_parameters())
    for name, p32 in ref32.named_parameters():
        p32 = p32.detach().double(); p64 = p64s[name].detach().double()
        pg = gpu_named[name].detach().cpu().double(); p0 = init[name].double()
        d = (pg - p64).abs()
        out = d > 1e-2 * lr + 1e-6 * p64.abs()
        keep = ~out
        e_hip = (pg - p64)[keep].norm().item(); e_cpu = (p32 - p64)[keep].norm().item()
        tol = 4 * e_cpu + 1e-4 * (p64 - p0).norm().item() + 1e-7 * p64.norm().item() + 1e-12
        print(f"{name:32s} n={p64.numel():7d} out={int(out.sum()):4d} e_hip={e_hip:.2e} e_cpu={e_cpu:.2e} tol={tol:.2e} ratio={e_hip/tol:.2f} upd={(p64-p0).norm().item():.2e}")


T.check_params = check
key = sys.argv[1] if len(sys.argv) > 1 else "G4/resnet222_c100_adam"
T.test_local_trainer_matches_oracle(key)
