#!/usr/bin/env python3
"""Headline benchmark: whole-node images/sec of the reference MNIST CNN (tf_dist_example.py)
with global batch 64*N on N MI355X GPUs (BASELINE.json metric/config).

    python bench.py                                   # N=1 (exactly one replica, cuda:0)
    python bench.py --gpus 8                          # self-launches 8 replica processes
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Runs the framework's training engine: MirroredStrategy over exactly N devices (one process per
GPU; RCCL / the xGMI all-reduce kernel between them) -> Keras Sequential exactly as the reference
builds it -> compile(SCCE from_logits, SGD 1e-3, SparseCategoricalAccuracy) -> the fused MI355X
engine's executions (hand-written gfx950 kernels, device-resident synthetic MNIST-shaped dataset
with map(scale).cache().shuffle(10000).batch(64*N).repeat(), hipGraph-captured executions incl.
the gradient all-reduce and the SGD update).  The timed loop drives the trainer's execution loop
(``run_train``, the loop ``Model.fit`` runs between callbacks) without progress-bar/log reads.
W untimed warm-up steps, then EXACTLY K timed steps bracketed by barrier + device sync (the clock
stops at each rank's closing device sync, before the closing barrier); the MAX time over ranks is
reported by rank 0 as one JSON line, together with a post-run check that the parameters are
bit-identical on every replica.  The first timed execution's input indices are prefetched before
the clock starts (input pipeline prefetch depth: one execution).

Without a launcher and N > 1 the script starts N-1 extra replica processes of itself before any
GPU call (MirroredStrategy(devices=[/gpu:0 .. /gpu:N-1])).  With TDL_SHARE_GPU=1 the N replicas
may share fewer physical GPUs (testing on a one-GPU box).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _spe(K: int, cap: int = 25) -> int:
    """Steps per execution: the largest divisor of K that is <= cap (one graph launch per
    execution; the timed region replays K / spe graphs).  Measured on one MI355X
    (profiles/mnist_bench_spe_sweep_r5.txt): at K=1000, 20-25 steps (40-50 kernel nodes) per graph
    run 0.5 % faster than 50; at K=20 one graph of 20 beats 2 x 10 / 4 x 5 (every graph launch
    costs the region its own submission latency); round 2's sweep put 100-1000 steps per graph
    5 % behind 50 (profiles/mnist_bench_spe_sweep_r2.txt)."""
    for d in range(min(K, cap), 0, -1):
        if K % d == 0:
            return d
    return 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--per-replica-batch", type=int, default=64)
    ap.add_argument("--steps-per-execution", type=int, default=0, help="0 = auto")
    ap.add_argument("--comm", choices=["auto", "nccl", "ring"], default="auto",
                    help="CollectiveCommunication: AUTO (xGMI kernel + RCCL), NCCL (RCCL only), RING (TCP)")
    ap.add_argument("--take", type=int, default=0, help="diagnostics: train on the first N images only")
    ap.add_argument("--mode", choices=["process", "single", "threads"], default="process",
                    help="N > 1 without a launcher: one replica process per GPU (default, the scaling mode), "
                         "or ONE process driving all N devices (TF's single-process MirroredStrategy: one host "
                         "thread launching every device's captured graph; 'threads' is an alias)")
    ap.add_argument("--engine", choices=["fused", "generic"], default="fused",
                    help="fused: the hand-written fused MNIST step (the headline); generic: the autograd engine "
                         "any model gets (TDL_DISABLE_FUSED=1) -- measures the cliff a model change meets")
    ap.add_argument("--variant", choices=["reference", "same", "dropout"], default="reference",
                    help="(generic engine) the reference CNN, with padding='same' convs, or with a Dropout layer")
    args = ap.parse_args()
    if args.engine == "generic":
        os.environ["TDL_DISABLE_FUSED"] = "1"
    elif args.variant != "reference":
        ap.error("--variant needs --engine generic (the fused engine runs the reference model only)")
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    import torch

    import tensorflow_distributed_learning_amd as tdl
    from tensorflow_distributed_learning_amd.data import tfds
    from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn
    from tensorflow_distributed_learning_amd.parallel import consistency
    from tensorflow_distributed_learning_amd.parallel.launch import ipc_mode

    world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if world and world != args.gpus:
        raise SystemExit(f"bench.py: launched with WORLD_SIZE={world} but --gpus {args.gpus}")
    # exactly N devices: on an 8-GPU node `--gpus 1` is ONE replica, `--gpus N` without a launcher
    # spawns the other N-1 replica processes here (no GPU has been touched yet)
    devices = [f"/gpu:{i}" for i in range(args.gpus)]
    # (spawn=True: one replica PROCESS per GPU -- the scaling mode -- when started without a launcher;
    # --mode single: one process for every device, engine/mirrored.py)
    single = args.mode in ("single", "threads") and args.gpus > 1 and not world
    strategy = tdl.distribute.MirroredStrategy(devices=devices, communication=args.comm.upper(), spawn=not single)
    R = strategy.num_replicas_in_sync
    if R != args.gpus:
        raise SystemExit(f"bench.py: strategy has {R} replicas, expected {args.gpus}")
    rank = strategy.extended.rank
    B = args.per_replica_batch * R
    K, W = args.steps, args.warmup
    spe = args.steps_per_execution or _spe(K)

    # synthetic MNIST-shaped data (no network): the reference's input pipeline
    (ds_all, info) = tfds.load("mnist", as_supervised=True, with_info=True)

    def scale(image, label):
        image = image.to(torch.float32)
        image = image / 255
        return image, label

    src = ds_all["train"].take(args.take) if args.take else ds_all["train"]
    train = src.map(scale).cache().shuffle(10000).batch(B).repeat()
    options = tdl.data.Options()
    options.experimental_distribute.auto_shard_policy = tdl.data.AutoShardPolicy.OFF
    train = train.with_options(options)

    def build():
        if args.variant == "reference":
            return build_mnist_cnn()
        L = tdl.keras.layers
        pad = "same" if args.variant == "same" else "valid"
        layers = [L.Conv2D(32, 3, activation="relu", padding=pad, input_shape=(28, 28, 1)), L.MaxPooling2D(),
                  L.Conv2D(64, 3, activation="relu", padding=pad), L.MaxPooling2D(), L.Flatten()]
        if args.variant == "dropout":
            layers.append(L.Dropout(0.25))
        return tdl.keras.Sequential(layers + [L.Dense(128, activation="relu"), L.Dense(10)])

    with strategy.scope():
        model = build()
        model.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tdl.keras.optimizers.SGD(learning_rate=0.001),
                      metrics=[tdl.keras.metrics.SparseCategoricalAccuracy()],
                      steps_per_execution=spe)
    trainer = model._get_trainer()
    handler = trainer.prepare(train) if hasattr(trainer, "prepare") else None
    if args.engine == "fused" and (trainer.kind != "fused" or handler is None):
        raise SystemExit(f"bench: fused MI355X engine not selected ({getattr(model, '_fused_reason', '?')})")
    if handler is None:
        if hasattr(trainer, "host_handler"):
            handler = trainer.host_handler(train)
        else:
            from tensorflow_distributed_learning_amd.engine.trainer import HostDataHandler

            handler = HostDataHandler(train, strategy)
        handler.new_iterator()
    comm = strategy.extended.communicator
    dev = strategy.extended.device

    def sync_all():
        if single:
            trainer.finish()  # every local device
        else:
            torch.cuda.synchronize(dev)

    fused = trainer.kind == "fused"
    if fused:
        trainer.warm_graphs(K)
    if W:
        if fused:
            trainer.warm_graphs(W)
        trainer.run_train(handler, W)
    if not fused and hasattr(trainer, "warm_graphs"):
        trainer.warm_graphs(K)  # generic engine: its execution graphs, captured once a step has run eagerly
    # input prefetch (depth one execution, as tf.data prefetch): the first timed execution's batch
    # indices are assembled and uploaded before the clock starts; later ones overlap the GPU
    if fused:
        trainer.prefetch(handler, K)
    sync_all()
    comm.barrier()
    sync_all()
    # (TDL_BENCH_EVENTS=1: device-side events around the steps, for the stderr diagnostics line)
    events = os.environ.get("TDL_BENCH_EVENTS", "0") == "1"
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    if events:
        ev0.record()
    done = trainer.run_train(handler, K)
    if events:
        ev1.record()
    t_host = time.perf_counter() - t0
    sync_all()
    dt = time.perf_counter() - t0
    # closing bracket: every rank's clock stopped at its own device sync; the barrier then only
    # joins the ranks (its latency is measurement overhead, not training work).  The MAX over ranks
    # below is the span from the earliest start to the last rank's finish (the in-graph all-reduce
    # of every step already keeps the ranks in lock step).
    comm.barrier()
    sync_all()
    print(f"timed region: wall {dt * 1e3:.3f} ms = host launch {t_host * 1e3:.3f} ms + device drain "
          f"{(dt - t_host) * 1e3:.3f} ms" + (f"; device events {ev0.elapsed_time(ev1):.3f} ms" if events else ""),
          file=sys.stderr)
    if done != K:
        raise SystemExit(f"bench: ran {done} steps instead of {K}")
    if single:
        per_rank = [dt]  # one process, one clock around every device's work
        logs = trainer.logs()
        identical = trainer.replicas_identical()
    else:
        t = torch.tensor([dt], dtype=torch.float64, device=dev if comm.name == "rccl" else "cpu")
        per_rank = [float(v) for v in comm.all_gather(t).reshape(-1).tolist()]
        dt = max(per_rank)
        logs = trainer.logs()  # also raises if an xGMI all-reduce timed out on this rank
        identical = consistency.replicas_identical(comm, trainer.W)
    ips = K * B / dt
    ht = getattr(trainer, "_host_times", None)
    if ht:
        import numpy as np

        a = np.array(ht[-max(1, K // max(1, spe)):]) * 1e6
        print(f"host us per execution (take, graph+upload, launch): median {np.median(a, 0).round(1).tolist()} "
              f"max {a.max(0).round(1).tolist()}", file=sys.stderr)
    from tensorflow_distributed_learning_amd.parallel import bucketing

    # modelled multi-GPU prediction (parallel/bucketing.py), from this run's step time at N = 1
    # and the recorded one-GPU number otherwise -- the driver's SCALE run checks it
    predicted = bucketing.predict_mnist_scaling(
        dt / K * 1e3 if R == 1 and args.per_replica_batch == 64 else bucketing.MNIST_T1_MS_RECORDED,
        twoshot_min_r=int(os.environ.get("TDL_FX_TWOSHOT_MIN_R", "3"))) if fused else None
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec (whole node) MNIST CNN global_batch=64*N",
            "value": round(ips, 1),
            "unit": "images/sec",
            "n_gpus": R,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(dt / K * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic MNIST-shaped (device-resident map(scale).cache().shuffle(10000).batch(64*N)); random init",
            "config": {"model": "tf_dist_example.py MNIST CNN (Conv32-Pool-Conv64-Pool-Dense128-Dense10, 225,034 params)",
                       "global_batch": B, "seq_len": None, "image_shape": [28, 28, 1],
                       "parallelism": f"dp{R}", "engine": trainer.kind, "communicator": comm.name,
                       "variant": args.variant,
                       "process_model": "single-process" if single else ("one process per GPU" if R > 1 else "single"),
                       # what actually ran: the communicator class (torch RCCL process group, the
                       # framework's own RCCL communicator, gloo + xGMI, local) and the HIP IPC mode
                       # every replica was started with (parallel/launch.py REPLICA_SHARED_ENV)
                       "communicator_impl": type(comm).__name__, "ipc_mode": ipc_mode(),
                       "allreduce": getattr(trainer, "allreduce_mode", None) or getattr(comm, "algorithm", comm.name),
                       "kernels_per_step": 2 if all(getattr(t, "_steps", None) and all(
                           getattr(st, "fused_bwd", False) for st in t._steps.values())
                           for t in getattr(trainer, "subs", [trainer])) else None,
                       "steps_per_execution": spe,
                       "graph_captured": bool(getattr(trainer, "capture", None) if fused else getattr(
                           trainer, "_graphs", None)),
                       "input_prefetch_executions": 1,
                       "allreduce_in_graph": bool(getattr(trainer, "capture_comm", False) and R > 1),
                       "replicas_identical": identical,
                       "final_loss": round(logs["loss"], 4),
                       # per-rank timed-region spread (the MAX is reported), and why any faster path
                       # was not taken on this job (self-tests, capture probes, xGMI set-up)
                       "rank_ms_per_step": [round(v / K * 1e3, 5) for v in per_rank],
                       "rank_spread_pct": round(100.0 * (max(per_rank) - min(per_rank)) / max(per_rank), 2),
                       "fallbacks": list(getattr(trainer, "fallbacks", [])) + (
                           [f"xgmi: {comm.xgmi_reason}"] if getattr(comm, "xgmi_reason", "") else [])},
            "predicted": predicted,
        }), flush=True)
    strategy.shutdown()
    if not identical:
        sys.exit(3)


if __name__ == "__main__":
    main()
