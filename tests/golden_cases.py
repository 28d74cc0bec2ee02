"""Load the committed golden vectors (tests/golden/*.json, produced from the reference by
tests/golden/make_golden.py) and rebuild their inputs."""
from __future__ import annotations

import functools
import json
import pathlib
import sys

GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(GOLDEN))

import synth_text  # noqa: E402
import gpt2_files  # noqa: E402

from inline_texts import INLINE  # noqa: E402


def input_bytes(spec) -> bytes:
    k = spec["kind"]
    if k == "fixture":
        return (gpt2_files.FIXTURES / spec["name"]).read_bytes()
    if k == "inline":
        return INLINE[spec["name"]].encode("utf-8")
    if k == "synth":
        text = synth_text.generate(spec["seed"], spec["n_chars"], spec["flavour"])
        assert synth_text.sha256_text(text) == spec["sha256"], "synthetic generator drifted"
        return text.encode("utf-8")
    if k == "string":
        return bytes.fromhex(spec["text_hex"])
    raise ValueError(k)


def names(prefix):
    return sorted(p.stem[len(prefix) + 1:] for p in GOLDEN.glob(f"{prefix}_*.json"))


@functools.lru_cache(maxsize=None)
def load(prefix, name):
    return json.loads((GOLDEN / f"{prefix}_{name}.json").read_text())


def train_expect(name):
    o = load("train", name)
    merges = [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in o["merges"]]
    vocab = {i: bytes.fromhex(h) for i, h in o["vocab"]}
    return o, vocab, merges


def tokenizer_inputs(o):
    """(vocab, merges) for an encode golden's tokenizer spec."""
    spec = o["tokenizer"]
    if spec == "gpt2":
        return gpt2_files.load_gpt2(o["special_tokens"])
    _, vocab, merges = train_expect(spec.split(":", 1)[1])
    return vocab, merges


def encode_text(o) -> str:
    spec = o["text"]
    return input_bytes(spec).decode("utf-8")
