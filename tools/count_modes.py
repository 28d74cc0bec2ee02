"""Count-kernel breakdown on the bench corpus in HBM: k_count2 device time per BPE355_COUNT_MODE
(run once per mode: the knob is read once per process).  Timing only."""
import ctypes, os, sys
sys.path[:0] = ["transformer-lm_amd", "."]
import torch
from bpe_amd import _lib, train_bpe_device
from bpe_amd.train import last_train_stats
n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 11_899_998_208
L = _lib.lib()
c = torch.empty(n, dtype=torch.uint8, device="cuda")
_lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(c.data_ptr()), n, 2, 0, 0, None), "synth")
torch.cuda.synchronize()
L.bpe_set_timing(1)
for i in range(3):
    train_bpe_device(c.data_ptr(), n, 256, ["<|endoftext|>"], keep_device_buffers=True)
    st = last_train_stats()
print(f"mode {os.environ.get('BPE355_COUNT_MODE', '0')}: k_count2 {st['count_kernel_ms']:.2f} ms, "
      f"reduce {st['count_reduce_ms']:.2f} ms, count phase {st['t_count_ms']:.2f} ms, records {st['n_count_records']}",
      flush=True)
