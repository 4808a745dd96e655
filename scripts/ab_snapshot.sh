#!/bin/bash
# Snapshot the current build (package + built extensions + bench / stamp scripts) into ab/<name>/ so that
# a later build can be A/B-benched against it in the SAME gpurun call (same box, interleaved runs):
#   bash scripts/ab_snapshot.sh base        # then change + rebuild, then on the GPU:
#   python ab/base/bench.py ...  vs  python bench.py ...
set -e
name=${1:?name}
dst=ab/$name
rm -rf "$dst"
mkdir -p "$dst/scripts"
cp -r tensorflow_distributed_learning_amd "$dst/"
find "$dst" -name __pycache__ -prune -exec rm -rf {} +
cp bench.py "$dst/"
cp scripts/stamps_mnist.py scripts/stamps_step.py "$dst/scripts/" 2>/dev/null || true
echo "snapshot $dst: $(du -sh $dst | cut -f1)"
