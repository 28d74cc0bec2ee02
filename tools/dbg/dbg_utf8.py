import sys, random
sys.path.insert(0, "transformer-lm_amd"); sys.path.insert(0, "tests")
import test_gpu_utf8 as T
import bpe_amd
from bpe_amd import _lib
_lib.require_device()
for s in [("中"*100).encode(), ("a"*15+"中"*100).encode(), ("é"*300).encode(), ("😀"*300).encode(), b"a"*40 + b"\xe4\xb8\xad"*30]:
    print(len(s), T._gpu_error_pos(s), T._cpu_error_pos(s))
rng = random.Random(100)
for it in range(12):
    n = rng.choice([40, 300, 2048, 5000])
    data = bytearray(T._text(rng, n))
    for _ in range(rng.choice([1, 1, 2])):
        anchor = rng.choice([16, 1024])
        p = min(len(data), max(0, rng.randrange(0, len(data) + 1) // anchor * anchor + rng.choice([-3, -2, -1, 0, 1, 2])))
        data[p:p] = rng.choice(T.BAD)
    data = bytes(data)
    print(it, len(data), T._gpu_error_pos(data), T._cpu_error_pos(data))
