"""Size- and topology-aware plan for the gradient all-reduce (README.md:21-23: the AUTO runtime
picks its algorithm "by hardware, network topology, tensor size"; TF's
``CommunicationOptions.bytes_per_pack`` splits gradients into packs of that size).

Model of one MI355X node (MI355X_MICROARCH.md): every GPU has 7 point-to-point xGMI links, about
153.6 GB/s per direction each, to the 7 other GPUs (a full mesh; no switch).  A ring all-reduce
moves ``2 (R-1)/R x bytes`` through every GPU; RCCL runs one ring channel per direct link, so at
R GPUs ``min(R-1, 7)`` links carry it in parallel and one ring alone would be bound by ONE link.
Each collective call also pays a fixed latency (launch + the ring's 2(R-1) dependent hops; a
modelled 25 us for RCCL, the measured 4.7 us for the xGMI one-shot kernel).

    t(bucket) = L + 2 (R-1)/R * bucket_bytes / (eff * 153.6 GB/s * min(R-1, 7))

With the gradient in K buckets the per-call latency costs K * L in total, while the first bucket
can only start once its gradients are final; the default plan therefore uses the smallest K >= 4
(overlap with backward) whose buckets are at least 4 MiB, unless ``bytes_per_pack`` is given.
For ResNet-50 (25.6 M params) at R = 8: 102 MB of f32 gradient in 4 buckets of ~25.6 MB, each
~68 us of wire time (+25 us latency) at eff = 0.6 -> ~0.37 ms of all-reduce per step to hide
behind a ~19 ms backward; with bf16 on the wire (``all_reduce_dtype="bfloat16"``) half that.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass
from typing import Optional

XGMI_LINK_GBPS = 153.6       # per direction, per link (MI355X_MICROARCH.md)
XGMI_LINKS = 7               # point-to-point links per GPU (8-GPU full mesh)
# Per-call fixed costs.  MEASURED on one MI355X (profiles/comm_fixed_costs_r4.jsonl,
# scripts/bench_comm_fixed.py, median of 7 interleaved repeats): the xGMI one-shot kernel between 2
# replica processes sharing the GPU costs 4.7 us at 64 KiB (flags, fences, launch; no fabric hop).  RCCL's per-call latency is NOT
# measurable on a one-GPU box (a world-1 RCCL all-reduce launches nothing: 0.07 us) and stays the
# modelled 25 us for 2(R-1) dependent ring hops on one node.  The link term is modelled too.
XGMI_CALL_US = 4.7           # measured (see above)
RCCL_CALL_LATENCY_US = 25.0  # modelled
LINK_EFFICIENCY = 0.6        # modelled achieved fraction of the link rate
MIN_BUCKET_BYTES = 4 << 20
MIN_BUCKETS = 4

DTYPE_BYTES = {"float32": 4, "bfloat16": 2, "float16": 2}


@dataclass
class BucketPlan:
    algorithm: str
    world: int
    local_world: int
    grad_numel: int
    wire_dtype: str
    wire_bytes: int
    n_buckets: int
    bucket_bytes: int
    links_used: int
    per_bucket_us: float
    total_us: float

    def as_dict(self) -> dict:
        d = asdict(self)
        d["per_bucket_us"] = round(self.per_bucket_us, 1)
        d["total_us"] = round(self.total_us, 1)
        xg = self.algorithm.startswith("xgmi")
        d["cost_model"] = {
            "per_bucket_us": "modelled",
            "call_latency_us": XGMI_CALL_US if xg else RCCL_CALL_LATENCY_US,
            "call_latency_source": "measured (profiles/comm_fixed_costs_r4.jsonl)" if xg else "modelled",
            "fabric": f"modelled: {XGMI_LINK_GBPS} GB/s per xGMI link x efficiency {LINK_EFFICIENCY}",
        }
        return d


def ring_allreduce_us(nbytes: int, world: int, links: Optional[int] = None) -> float:
    """Modelled time of one ring all-reduce of ``nbytes`` over the node's xGMI mesh."""
    if world <= 1:
        return 0.0
    links = links if links is not None else min(world - 1, XGMI_LINKS)
    bw = LINK_EFFICIENCY * XGMI_LINK_GBPS * 1e9 * links
    return RCCL_CALL_LATENCY_US + 2.0 * (world - 1) / world * nbytes / bw * 1e6


def xgmi_oneshot_us(nbytes: int, world: int) -> float:
    """Time of one xGMI one-shot all-reduce: the measured fixed cost + every rank pulling the
    ``nbytes`` of each peer over its own direct link, all links in parallel (modelled)."""
    if world <= 1:
        return 0.0
    return XGMI_CALL_US + nbytes / (LINK_EFFICIENCY * XGMI_LINK_GBPS * 1e9) * 1e6


XGMI_TWOSHOT_CALL_US = 6.8  # measured like XGMI_CALL_US (two flag rounds)
MNIST_GRAD_BYTES = 225_034 * 4
MNIST_T1_MS_RECORDED = 0.02562  # the driver's BENCH_r05 record (K=20, one MI355X)


def predict_mnist_scaling(t1_ms: float, ns=(2, 4, 8), twoshot_min_r: int = 3) -> dict:
    """MODELLED weak-scaling prediction for the reference CNN's exchange-in-finalize step, written
    before any multi-GPU measurement so the first SCALE run shows whether the fabric behaves as
    assumed.  Per step at N GPUs: the one-GPU step ``t1`` + the exchange's fixed cost (the measured
    one-/two-shot call cost, profiles/comm_fixed_costs_r4.jsonl: flags, fences, no fabric hop) + the
    fabric term: one-shot pulls every peer's whole 900 KB slab over that peer's link (all links in
    parallel: n / link), two-shot pulls a 1/N shard from every peer twice (2 n / N per link), at
    ``LINK_EFFICIENCY`` x 153.6 GB/s.  It ignores the overlap of the exchange with the finalize's own
    reduction work (pessimistic) and any contention inside a GPU (optimistic)."""
    bw = LINK_EFFICIENCY * XGMI_LINK_GBPS * 1e9  # bytes/s per link
    out_ms, eff = {}, {}
    for n in ns:
        if n <= 1:
            continue
        if n >= twoshot_min_r:
            extra_us = XGMI_TWOSHOT_CALL_US + 2.0 * (MNIST_GRAD_BYTES / n) / bw * 1e6
        else:
            extra_us = XGMI_CALL_US + MNIST_GRAD_BYTES / bw * 1e6
        t = t1_ms + extra_us * 1e-3
        out_ms[str(n)] = round(t, 5)
        eff[str(n)] = round(t1_ms / t, 3)
    return {"label": "modelled, not measured", "t1_ms": round(t1_ms, 5), "ms_per_step": out_ms,
            "scaling_efficiency": eff,
            "assumptions": {"link_GBps": XGMI_LINK_GBPS, "link_efficiency": LINK_EFFICIENCY,
                            "oneshot_fixed_us": XGMI_CALL_US, "twoshot_fixed_us": XGMI_TWOSHOT_CALL_US,
                            "grad_bytes": MNIST_GRAD_BYTES, "twoshot_from_n": twoshot_min_r}}


def plan(grad_numel: int, world: int, local_world: Optional[int] = None, wire_dtype: str = "float32",
         bytes_per_pack: int = 0, algorithm: str = "rccl") -> BucketPlan:
    """Bucket plan for a flat gradient of ``grad_numel`` elements on ``world`` replicas."""
    if wire_dtype not in DTYPE_BYTES:
        raise ValueError(f"all-reduce dtype must be one of {sorted(DTYPE_BYTES)}, got {wire_dtype!r}")
    local_world = world if local_world is None else local_world
    wire_bytes = grad_numel * DTYPE_BYTES[wire_dtype]
    if bytes_per_pack > 0:
        bucket = int(bytes_per_pack)
    else:
        k = MIN_BUCKETS
        while k > 1 and wire_bytes / k < MIN_BUCKET_BYTES:
            k -= 1
        bucket = -(-wire_bytes // k)
    bucket = max(1, min(bucket, wire_bytes))
    n = max(1, -(-wire_bytes // bucket))
    links = min(max(local_world - 1, 1), XGMI_LINKS)
    per = xgmi_oneshot_us(bucket, world) if algorithm.startswith("xgmi") else ring_allreduce_us(bucket, world, links)
    return BucketPlan(algorithm, world, local_world, grad_numel, wire_dtype, wire_bytes, n, bucket, links, per,
                      per * n if world > 1 else 0.0)
