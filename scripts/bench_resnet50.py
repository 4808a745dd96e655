#!/usr/bin/env python3
"""ResNet-50 training throughput (BASELINE configs 4/5): synthetic ImageNet-shaped data, random init,
Keras ResNet50 built with this framework, mixed_bfloat16 policy, SGD momentum 0.9, MirroredStrategy
(one process per GPU, RCCL bucketed all-reduce overlapped with backward).

    python scripts/bench_resnet50.py [--batch 256] [--steps 20] [--warmup 5]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 scripts/bench_resnet50.py

    python scripts/bench_resnet50.py --gpus 8                      # config 4, self-launched replicas
    python scripts/bench_resnet50.py --strategy mwms --workers 2 --gpus 8   # config 5 (2 tasks x 4 GPUs)

Prints one JSON line (rank 0) in the bench.py format.  ``--strategy mwms`` without a TF_CONFIG in
the environment starts ``--workers`` TF_CONFIG tasks on this node through the launcher
(``launch_local_workers``: every task sees every GPU and pins its replicas to disjoint devices,
so the xGMI all-reduce kernel and RCCL peer-to-peer work across tasks).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256, help="per-replica batch")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--dtype", default="mixed_bfloat16", choices=["mixed_bfloat16", "float32"])
    ap.add_argument("--gpus", type=int, default=1, help="replicas (GPUs) in the whole job")
    ap.add_argument("--workers", type=int, default=2, help="--strategy mwms: TF_CONFIG tasks on this node")
    ap.add_argument("--comm", choices=["auto", "nccl", "ring"], default="auto")
    ap.add_argument("--allreduce-dtype", choices=["float32", "bfloat16"], default="float32",
                    help="gradient dtype on the wire (CommunicationOptions.all_reduce_dtype)")
    ap.add_argument("--bytes-per-pack", type=int, default=0,
                    help="all-reduce bucket bytes (CommunicationOptions.bytes_per_pack; 0 = size/topology plan)")
    ap.add_argument("--conv-search", type=int, default=1,
                    help="1: MIOpen find-mode solver search per conv shape (torch.backends.cudnn.benchmark)")
    ap.add_argument("--strategy", default="mirrored", choices=["mirrored", "mwms"],
                    help="mwms: MultiWorkerMirroredStrategy over TF_CONFIG workers (BASELINE config 5)")
    args = ap.parse_args()

    if args.strategy == "mwms" and not os.environ.get("TF_CONFIG") and "WORLD_SIZE" not in os.environ:
        # BASELINE config 5 on one node: K TF_CONFIG tasks x G GPUs each, started here (no GPU
        # has been touched in this process)
        from tensorflow_distributed_learning_amd.parallel.launch import launch_local_workers

        if args.gpus % args.workers:
            ap.error("--gpus must be a multiple of --workers")
        sys.exit(launch_local_workers([sys.executable] + sys.argv, args.workers, args.gpus // args.workers))

    import torch

    import tensorflow_distributed_learning_amd as tdl

    torch.backends.cudnn.benchmark = bool(args.conv_search)
    tdl.keras.mixed_precision.set_global_policy(args.dtype)
    copts = tdl.distribute.experimental.CommunicationOptions(
        implementation=args.comm.upper(), bytes_per_pack=args.bytes_per_pack,
        all_reduce_dtype=None if args.allreduce_dtype == "float32" else args.allreduce_dtype)
    if args.strategy == "mwms":
        strategy = tdl.distribute.MultiWorkerMirroredStrategy(communication_options=copts)
    else:
        strategy = tdl.distribute.MirroredStrategy(devices=[f"/gpu:{i}" for i in range(args.gpus)],
                                                   communication_options=copts, spawn=True)
    R = strategy.num_replicas_in_sync
    if R != args.gpus:
        raise SystemExit(f"bench_resnet50: strategy has {R} replicas, expected --gpus {args.gpus}")
    dev = strategy.extended.device
    b = args.batch
    B = b * R
    # device-resident synthetic ImageNet-shaped dataset: 4 distinct global batches, repeated
    g = torch.Generator(device="cpu").manual_seed(0)
    n = 4 * B
    x = torch.empty(n, args.image, args.image, 3, dtype=torch.float32, device=dev)
    x.uniform_(0, 1)
    y = torch.randint(0, args.classes, (n,), generator=g).to(torch.int64).to(dev)
    ds = tdl.data.Dataset.from_tensor_slices((x, y)).batch(B, drop_remainder=True).repeat()
    opts = tdl.data.Options()
    opts.experimental_distribute.auto_shard_policy = tdl.data.AutoShardPolicy.OFF
    ds = ds.with_options(opts)

    with strategy.scope():
        model = tdl.keras.applications.ResNet50(weights=None, classes=args.classes, classifier_activation=None,
                                                input_shape=(args.image, args.image, 3))
        model.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tdl.keras.optimizers.SGD(learning_rate=0.01, momentum=0.9),
                      metrics=["sparse_categorical_accuracy"])
    trainer = model._get_trainer()
    handler = trainer.prepare(ds) if hasattr(trainer, "prepare") else None
    if handler is None:
        from tensorflow_distributed_learning_amd.engine.trainer import HostDataHandler

        handler = HostDataHandler(ds, strategy)
    comm = strategy.extended.communicator

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    if hasattr(trainer, "warm_graphs"):
        trainer.warm_graphs(args.steps)
    if os.environ.get("TDL_TRACE_LOSS") == "1":  # per-step loss of the warm-up steps (diagnostic)
        for i in range(args.warmup):
            trainer.reset_metrics()
            trainer.run_train(handler, 1)
            print(f"warmup step {i}: loss {trainer.logs()['loss']:.4f}", flush=True)
    else:
        trainer.run_train(handler, args.warmup)
    trainer.reset_metrics()  # the reported loss covers the timed steps only
    sync()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    done = trainer.run_train(handler, args.steps)
    sync()
    comm.barrier()
    sync()
    dt = time.perf_counter() - t0
    assert done == args.steps, done
    t = torch.tensor([dt], dtype=torch.float64, device=dev if comm.name == "rccl" else "cpu")
    comm.all_reduce(t, "max")
    dt = float(t.item())
    logs = trainer.logs()
    from tensorflow_distributed_learning_amd.parallel import consistency

    identical = consistency.replicas_identical(comm, trainer.W)
    if strategy.extended.rank == 0:
        print(json.dumps({
            "metric": "images/sec (whole node) ResNet-50 synthetic ImageNet-shaped",
            "value": round(args.steps * B / dt, 1), "unit": "images/sec", "n_gpus": R,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if args.dtype == "mixed_bfloat16" else "fp32",
            "data": "synthetic ImageNet-shaped, device-resident; random init",
            "config": {"model": "keras.applications.ResNet50 (25.6M params)", "global_batch": B,
                       "image": args.image, "parallelism": f"dp{R}", "strategy": type(strategy).__name__,
                       "workers": (len(strategy.extended.tf_config.cluster.training_tasks())
                                   if getattr(strategy.extended, "tf_config", None) else 1),
                       "engine": trainer.kind, "communicator": comm.name,
                       "allreduce": getattr(comm, "algorithm", comm.name),
                       # what ran (no modelled terms): bucket count / size / wire dtype of the all-reduce
                       "buckets": ({"n": trainer.plan.n_buckets if trainer._buckets is not None else 1,
                                    "bytes": trainer.plan.bucket_bytes, "wire_dtype": trainer.plan.wire_dtype,
                                    "overlapped_with_backward": trainer._buckets is not None}
                                   if R > 1 and getattr(trainer, "plan", None) else None),
                       "replicas_identical": identical, "final_loss": round(logs["loss"], 4)},
        }), flush=True)
    if strategy.extended.rank == 0:
        from tensorflow_distributed_learning_amd.ops import conv as _conv

        ch = _conv.choices()
        print(f"conv autotune: {sum(v == 'hip' for v in ch.values())}/{len(ch)} (shape, direction) pairs on the "
              f"hand-written kernels: {sorted(k[0] + str(k[1][1:]) + str(k[2]) for k, v in ch.items() if v == 'hip')}",
              file=sys.stderr, flush=True)
    strategy.shutdown()


if __name__ == "__main__":
    main()
