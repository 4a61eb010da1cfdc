import glob
import json
import os

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
STAT_KEYS = ("gen", "recv", "fwd", "sent", "processed", "peers", "sockets")


def names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(HERE, "*.npz")))


def load(name):
    z = np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["params"] = json.loads(str(d["params"]))
    return d
