import glob
import hashlib
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


def links_digest(a, b):
    """SHA-256 over the uint32 key arrays: pins link sets too large to commit."""
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(a, np.uint32).tobytes())
    h.update(np.ascontiguousarray(b, np.uint32).tobytes())
    return h.hexdigest()
