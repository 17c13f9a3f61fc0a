"""Golden vectors for the reference's weight hash (model/tensorflow/model.py:
172-177: sum over Keras get_weights() of md5(str(weight).encode("utf-8"))).

Run in the development container (python3 with torch builds the weights; the
digests are taken under /opt/conda/bin/python3.9, numpy 1.26.4, the same
print rules as the reference's pinned numpy 1.24.3):

    python3 tests/golden/make_weight_hash.py

str() of an array is numpy's summarised print form, so the expected digests
depend on the numpy version's array printing; the test checks that this
repo's reference_hash under the runtime numpy reproduces the legacy-numpy
digests.  TensorFlow is absent: the Keras get_weights() order itself is
restated (weights.keras_order), parity unpinned against TF.

Output: tests/golden/weight_hash.json (data only).
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "custom-alphazero_amd"))
from custom_alphazero.model.weights import init_weights, keras_order, weight_spec  # noqa: E402

LEGACY = "/opt/conda/bin/python3.9"
DIGEST = r"""
import hashlib, json, sys
import numpy as np
assert np.__version__.startswith("1.")
z = np.load(sys.argv[1], allow_pickle=False)
names = json.loads(sys.argv[2])
print(json.dumps([hashlib.md5(str(z[n]).encode("utf-8")).hexdigest() for n in names]))
"""

CASES = {
    "c4_seed0": dict(shape=(6, 7, 7, 4), seed=0, randomize_bn=False),
    "c4_seed3_bn": dict(shape=(6, 7, 7, 4), seed=3, randomize_bn=True),
    "c5_9x9_seed1": dict(shape=(9, 9, 9, 4), seed=1, randomize_bn=False),
}


def main():
    out = {}
    for case, c in CASES.items():
        H, W, A, C = c["shape"]
        spec = weight_spec(H, W, A, in_channels=C)
        w = init_weights(spec, seed=c["seed"], randomize_bn=c["randomize_bn"])
        names = keras_order(spec)
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "w.npz")
            np.savez(path, **w)
            digests = json.loads(subprocess.run([LEGACY, "-c", DIGEST, path, json.dumps(names)],
                                                check=True, capture_output=True, text=True).stdout)
        out[case] = {**c, "names": names, "md5": digests,
                     "hash": str(sum(int(d, 16) for d in digests))}
    with open(os.path.join(REPO, "tests", "golden", "weight_hash.json"), "w") as fp:
        json.dump(out, fp, indent=1)


if __name__ == "__main__":
    main()
