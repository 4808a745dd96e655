"""Bisect the generic engine's step by per-op checksums (utils/checksums.py).

    python scripts/diag_checksums.py run F out.json [steps]     # one training run, checksums dumped
    python scripts/diag_checksums.py compare a.json b.json      # first entry whose bits differ

Model / data / optimizer: scripts/diag_bnfuse.py (ResNet-style bottleneck blocks, bf16, BN, SGD
momentum 0.9, eager steps).  ``TDL_DETERMINISTIC=1`` also turns on
``torch.use_deterministic_algorithms`` (warn-only: every non-deterministic torch op is named on
stderr).
"""
import json
import os
import sys
import warnings

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def run(cfg, out, steps):
    os.environ["TDL_DEBUG_CHECKSUMS"] = "1"
    import torch

    if os.environ.get("TDL_DETERMINISTIC") == "1":
        torch.use_deterministic_algorithms(True, warn_only=True)
        warnings.simplefilter("always")
    from diag_bnfuse import run as run_model

    from tensorflow_distributed_learning_amd.utils import checksums as ck

    ck.enable(True)
    ck.reset()
    flags = {"F": (False, False, False), "T": (True, True, True)}[cfg]
    m = run_model(*flags, steps)
    torch.cuda.synchronize()
    rec = ck.dump(out)
    print(f"recorded {len(rec)} checksums -> {out}; weights sum {sum(float(abs(w).sum()) for w in m.get_weights()):.9e}",
          flush=True)


def compare(a_path, b_path, show=12):
    a, b = json.load(open(a_path)), json.load(open(b_path))
    from tensorflow_distributed_learning_amd.utils.checksums import first_difference

    d = first_difference(a, b)
    if d is None:
        print(f"IDENTICAL ({len(a)} checksums)")
        return 0
    i = d[0]
    print(f"FIRST DIFFERENCE at #{i}/{len(a)}: {d[1]} vs {d[2]}")
    for j in range(max(0, i - 2), min(len(a), len(b), i + show)):
        x, y = a[j], b[j]
        rel = abs(x["sum"] - y["sum"]) / max(abs(x["abs"]), 1e-30)
        mark = "  " if x["hash"] == y["hash"] else "!!"
        print(f"{mark} #{j:4d} {x['tag'][:60]:60s} sum {x['sum']:+.9e} vs {y['sum']:+.9e}  rel {rel:.2e}")
    ndiff = sum(1 for x, y in zip(a, b) if x["hash"] != y["hash"])
    print(f"{ndiff} of {min(len(a), len(b))} entries differ")
    return 1


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3], int(sys.argv[4]) if len(sys.argv) > 4 else 2)
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
