"""bpe_amd -- MI355X-native byte-level BPE, drop-in for gashon/transformer-lm's tokenizer path.

    from bpe_amd import train_bpe, Tokenizer, Vocab

mirror reference models/tokenizer/{train.py, tokenizer.py, vocab.py}.  Compute runs in
libbpe355.so (HIP, gfx950); there is no CPU fallback.
"""
from .train import (train_bpe, train_bpe_bytes, train_bpe_device, last_train_stats,  # noqa: F401
                    set_num_gpus, num_gpus, release_device_memory)
from .vocab import Vocab  # noqa: F401
from .tokenizer import Tokenizer  # noqa: F401
