"""tf.keras.mixed_precision: 'float32' or 'mixed_bfloat16' (bf16 compute, f32 master weights)."""
from __future__ import annotations

from . import models as _models


class Policy:
    def __init__(self, name: str):
        if name not in ("float32", "mixed_bfloat16", "mixed_float16", "bfloat16"):
            raise ValueError(f"unsupported dtype policy {name!r}")
        self.name = "mixed_bfloat16" if name in ("mixed_float16", "bfloat16") else name

    @property
    def compute_dtype(self):
        return "bfloat16" if self.name == "mixed_bfloat16" else "float32"

    @property
    def variable_dtype(self):
        return "float32"

    def __repr__(self):
        return f'<Policy "{self.name}">'


def set_global_policy(policy):
    p = policy if isinstance(policy, Policy) else Policy(policy)
    _models._GLOBAL_POLICY[0] = p.name


def global_policy() -> Policy:
    return Policy(_models._GLOBAL_POLICY[0])
