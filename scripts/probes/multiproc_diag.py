import json, os, subprocess, sys, textwrap, tempfile, numpy as np
ROOT = "/root/repo"
BODY = """
import json, os, sys, numpy as np, torch
import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn
from tensorflow_distributed_learning_amd.data.tfds import synthetic_mnist
out, lr = sys.argv[1], float(sys.argv[2])
strategy = tdl.distribute.MirroredStrategy(communication="RING")
R = strategy.num_replicas_in_sync
tdl.keras.utils.set_random_seed(5)
x, y = synthetic_mnist(2048, 2)
ds = tdl.data.Dataset.from_tensor_slices((x.reshape(-1, 28, 28, 1), y))
ds = ds.map(lambda i, l: (i.to(torch.float32) / 255, l)).cache().shuffle(2048, seed=9).batch(128).repeat()
with strategy.scope():
    m = build_mnist_cnn()
    m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tdl.keras.optimizers.SGD(lr), metrics=["sparse_categorical_accuracy"], steps_per_execution=4)
h = m.fit(ds, epochs=2, steps_per_epoch=8, verbose=0)
w = np.concatenate([v.ravel() for v in m.get_weights()])
np.save(os.path.join(out, f"w{strategy.extended.rank}_{R}_{lr}.npy"), w)
json.dump(h.history["loss"], open(os.path.join(out, f"l{strategy.extended.rank}_{R}_{lr}.json"), "w"))
"""
d = tempfile.mkdtemp()
open(f"{d}/job.py", "w").write(textwrap.dedent(BODY))
env = dict(os.environ, PYTHONPATH=ROOT, TDL_SHARE_GPU="1")
for lr in ("0.1", "0.01"):
    for n in (1, 2):
        r = subprocess.run([sys.executable, "-m", "tensorflow_distributed_learning_amd.launch", "--nproc-per-node", str(n), f"{d}/job.py", d, lr], env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-2000:]
    w1, w2 = np.load(f"{d}/w0_1_{lr}.npy"), np.load(f"{d}/w0_2_{lr}.npy")
    l1, l2 = json.load(open(f"{d}/l0_1_{lr}.json")), json.load(open(f"{d}/l0_2_{lr}.json"))
    print(f"lr={lr}: max|dw|={np.abs(w1-w2).max():.2e} (|w| max {np.abs(w1).max():.2f}) loss R1 {l1} R2 {l2}")
