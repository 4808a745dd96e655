import time, sys
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
import numpy as np, torch
import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.data import tfds, device as DD
(ds_all, info) = tfds.load("mnist", as_supervised=True, with_info=True)
def scale(image, label):
    return image.to(torch.float32) / 255, label
train = ds_all["train"].map(scale).cache().shuffle(10000).batch(64).repeat()
opts = tdl.data.Options(); opts.experimental_optimization.device_resident = True
lp = DD.lower(train.with_options(opts))
print("lowered", lp is not None)
st = DD.IndexStream(lp, None)
worst = (0, 0)
t0 = time.perf_counter()
for i in range(2000):
    t = time.perf_counter(); st.next_batch(); d = time.perf_counter() - t
    if d > worst[0]: worst = (d, i)
print("total ms", (time.perf_counter()-t0)*1e3, "worst ms", worst[0]*1e3, "at", worst[1])
# epoch generation alone, native vs the pure-Python fallback
from tensorflow_distributed_learning_amd.data import dataset as D
for k in range(3):
    t = time.perf_counter(); D._shuffle_indices(60000, 10000, np.random.default_rng(k)); print("native shuffle ms", (time.perf_counter() - t) * 1e3)
print("native module", D._native_or_none())
