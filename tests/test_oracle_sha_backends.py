"""The C oracle's SHA-256 has two backends (oracle/fri_oracle.c): the portable
restatement of FIPS 180-4 and the x86 SHA extensions, which the reference's
sha2 0.10.8 also selects at run time on CPUs that have them (the GPU box's
EPYC does; ORC_NO_SHANI=1 forces the portable one).  Both must give hashlib's
digests, and a whole commit transcript must not depend on the backend."""
import ctypes
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import ctypes, hashlib, json, os, random, sys
sys.path.insert(0, os.path.join(sys.argv[1], "oracle"))
import numpy as np
import fri_oracle as fo
lib = fo.load_c_oracle()
f = lib.orc_sha256
random.seed(7)
bad = 0
for n in list(range(0, 160)) + [1000, 4096, 65536 + 3]:
    m = bytes(random.getrandbits(8) for _ in range(n))
    out = ctypes.create_string_buffer(32)
    f(m, n, out)
    bad += out.raw != hashlib.sha256(m).digest()
L = 14
d = (1 << L) >> 3
c = np.ascontiguousarray(fo.splitmix64_np(3, d))
och = fo.OrcChannel(); lib.orc_channel_init(ctypes.byref(och)); res = fo.OrcFriResult()
assert lib.orc_fri_commit_fast(c.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), d, L, 5, 5, fo.P,
                               ctypes.byref(och), None, ctypes.byref(res), None, None) == 0
print(json.dumps({"backend": lib.orc_sha_backend(), "bad": bad,
                  "roots": [bytes(res.roots[k]).hex() for k in range(res.n_layers)], "state": och.state.decode()}))
"""


def _run(no_shani):
    env = dict(os.environ)
    env.pop("ORC_NO_SHANI", None)
    if no_shani:
        env["ORC_NO_SHANI"] = "1"
    out = subprocess.run([sys.executable, "-c", _CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_sha_backends_agree_with_hashlib_and_each_other():
    fast, port = _run(False), _run(True)
    assert port["backend"] == 0
    assert fast["bad"] == 0 and port["bad"] == 0
    assert fast["roots"] == port["roots"] and fast["state"] == port["state"]
    # on an x86 host with the SHA extensions the default is the extension backend
    flags = open("/proc/cpuinfo").read() if os.path.exists("/proc/cpuinfo") else ""
    if " sha_ni" in flags:
        assert fast["backend"] == 1
