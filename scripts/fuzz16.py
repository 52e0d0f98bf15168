"""Randomized GF(2^16) plan fuzz on the GPU against the NumPy oracle: k, m, widths, batches, fused
copies, scattered rows, column windows and engines drawn at random (SEED, N from the environment).
One line per case, then the count of wrong ones; exit 1 if any. PYTHONPATH=. python scripts/fuzz16.py"""
import numpy as np, torch, sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gpu_rscode_amd import alloc_rows, gf
from gpu_rscode_amd.ops import Gemm16Plan, GemmPlan


def main():
    F = gf.field(16)
    rng = np.random.default_rng(int(os.environ.get("SEED", "1")))
    bad = 0
    for case in range(int(os.environ.get("N", "60"))):
        k = int(rng.integers(1, 420)); m = int(rng.integers(1, 70))
        C = int(rng.integers(1, 40000)) * 2
        B = int(rng.choice([1, 1, 1, 2, 5]))
        copies = bool(rng.integers(0, 2))
        scattered = bool(rng.integers(0, 2)) and B == 1
        engine = str(rng.choice(["mfma", "auto", "valu16"]))
        coeff = rng.integers(0, 65536, size=(m, k))
        if B == 1:
            x = alloc_rows(k, C, "cuda"); x.copy_(torch.from_numpy(rng.integers(0, 256, (k, C), dtype=np.uint8)))
            ins = [x[i].clone() for i in range(k)] if scattered else x
            y = alloc_rows(m, C, "cuda", fill=0x33)
            z = alloc_rows(k, C, "cuda", fill=0) if copies else None
            cp = [z[i] if i % 3 else None for i in range(k)] if copies else None
            try:
                plan = Gemm16Plan(ins, y, coeff, copies=cp, engine=engine)
            except ValueError as e:
                print(f"skip k={k} m={m} C={C} B={B} engine={engine}: {e}", flush=True)
                continue
            c0 = int(rng.integers(0, C // 2)) * 2 if rng.integers(0, 3) == 0 else 0
            n = int(rng.integers(0, (C - c0) // 2 + 1)) * 2 if c0 else C
            plan.run(col0=c0, ncols=n)
            torch.cuda.synchronize()
            want = F.gemm(coeff, np.ascontiguousarray(x.cpu().numpy()).view("<u2"))
            got = y.cpu().numpy().view("<u2")
            s0, s1 = c0 // 2, (c0 + n) // 2
            ok = np.array_equal(got[:, s0:s1], want[:, s0:s1]) and (got[:, :s0] == 0x3333).all() and (got[:, s1:] == 0x3333).all()
            if copies:
                zz, xx = z.cpu().numpy(), x.cpu().numpy()
                ok = ok and all(np.array_equal(zz[i, c0:c0 + n], xx[i, c0:c0 + n]) for i in range(k) if i % 3)
        else:
            x = torch.from_numpy(rng.integers(0, 256, (B, k, C), dtype=np.uint8)).cuda()
            y = torch.zeros((B, m, C), dtype=torch.uint8, device="cuda")
            try:
                plan = Gemm16Plan(x, y, coeff, engine=engine)
            except ValueError as e:
                print(f"skip k={k} m={m} C={C} B={B} engine={engine}: {e}", flush=True)
                continue
            plan.run()
            torch.cuda.synchronize()
            xh = x.cpu().numpy(); yh = y.cpu().numpy()
            ok = all(np.array_equal(yh[b].view("<u2"), F.gemm(coeff, np.ascontiguousarray(xh[b]).view("<u2"))) for b in range(B))
        tag = f"k={k} m={m} C={C} B={B} copies={copies} scattered={scattered} engine={engine}->{plan.engine}"
        if not ok:
            bad += 1
            print("BAD", tag, flush=True)
        else:
            print("ok ", tag, flush=True)
    print("bad", bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
