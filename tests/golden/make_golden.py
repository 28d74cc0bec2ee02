"""Regenerate the golden vectors in tests/golden/*.json from the REFERENCE implementation.

Runs only in the build container, where the reference is mounted read-only at
/root/reference; it imports the reference's own modules (models/tokenizer/train.py,
tokenizer.py) and records their outputs as data.  Nothing here is needed at test time:
the tests read the committed JSON files.

    python tests/golden/make_golden.py [--only NAME ...]

Every case records its input spec (a fixture file name, inline text, or a synth_text.py
recipe + sha256), the arguments, and the reference's output:
  train:  ordered merges (hex bytes pairs) and the exact id->bytes vocab,
  words:  the pretoken->count table of extract_subword_frequencies (train.py:16-28),
  encode: the id list of Tokenizer.encode (tokenizer.py:111-138).
"""
from __future__ import annotations

import argparse
import io
import json
import logging
import os
import pathlib
import sys
import tempfile
import time
import contextlib

HERE = pathlib.Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF = pathlib.Path("/root/reference")
sys.dont_write_bytecode = True
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(REPO / "tests"))

import synth_text  # noqa: E402
import gpt2_files  # noqa: E402

EOT = "<|endoftext|>"

# ---------------------------------------------------------------------------------------
# inputs
from inline_texts import INLINE  # noqa: E402


def synth_spec(seed, n, flavour):
    return {"kind": "synth", "seed": seed, "n_chars": n, "flavour": flavour}


def input_text(spec) -> str:
    k = spec["kind"]
    if k == "fixture":
        return (gpt2_files.FIXTURES / spec["name"]).read_bytes().decode("utf-8")
    if k == "inline":
        return INLINE[spec["name"]]
    if k == "synth":
        return synth_text.generate(spec["seed"], spec["n_chars"], spec["flavour"])
    raise ValueError(k)


def input_bytes(spec) -> bytes:
    if spec["kind"] == "fixture":
        return (gpt2_files.FIXTURES / spec["name"]).read_bytes()
    return input_text(spec).encode("utf-8")


def fixture(name):
    return {"kind": "fixture", "name": name}


def inline(name):
    return {"kind": "inline", "name": name}


TRAIN_CASES = [
    ("corpus_en_500", fixture("corpus.en"), 500, [EOT]),
    ("corpus_en_1000", fixture("corpus.en"), 1000, [EOT]),
    ("corpus_en_2500_nospecial", fixture("corpus.en"), 2500, []),
    ("tiny_400", fixture("tinystories_sample.txt"), 400, [EOT]),
    ("tiny_1200", fixture("tinystories_sample.txt"), 1200, [EOT]),
    ("tiny_3000", fixture("tinystories_sample.txt"), 3000, [EOT]),
    ("edge_empty", inline("empty"), 300, [EOT]),
    ("edge_abc", inline("abc"), 270, []),
    ("edge_crlf", inline("crlf"), 300, []),
    ("edge_aaaa", inline("aaaa"), 300, []),
    ("edge_special_word", inline("special_word"), 320, [" the", "hello", EOT]),
    ("edge_dup_special", inline("dup_special"), 300, ["a", EOT, EOT]),
    ("edge_ws", inline("ws_edges"), 290, []),
    ("edge_contractions", inline("contractions"), 300, []),
    ("edge_below_base", fixture("corpus.en"), 100, [EOT]),
    ("synth_mixed_200k", synth_spec(1, 200_000, "mixed"), 1000, [EOT]),
    ("synth_space_100k", synth_spec(3, 100_000, "space"), 700, [EOT]),
    ("synth_ascii_1m", synth_spec(2, 1_000_000, "ascii"), 1000, [EOT]),
    ("synth_ascii_4m", synth_spec(4, 4_000_000, "ascii"), 2000, [EOT]),
]

WORD_CASES = [
    ("corpus_en", fixture("corpus.en"), [EOT]),
    ("tiny", fixture("tinystories_sample.txt"), [EOT]),
    ("crlf", inline("crlf"), []),
    ("special_word", inline("special_word"), [" the", "hello", EOT]),
    ("ws_edges", inline("ws_edges"), []),
    ("contractions", inline("contractions"), []),
    ("synth_mixed_200k", synth_spec(1, 200_000, "mixed"), [EOT]),
    ("synth_space_100k", synth_spec(3, 100_000, "space"), [EOT]),
]

ENCODE_STRINGS = [
    "",
    "s",
    "\U0001F643",
    "Hello, how are you?",
    "Héllò hôw are ü? \U0001F643",
    "Héllò hôw <|endoftext|><|endoftext|> are ü? \U0001F643<|endoftext|>",
    "Hello, how <|endoftext|><|endoftext|> are you?<|endoftext|>",
    "trailing spaces   ",
    "  \n\n lead and\tmixed 　 ws\r\nwith CRLF\r",
    "<|endoftext|>",
    "<|endoftext|x <|endoftext|><|endoftext|",
]

# (tokenizer spec, specials, text spec)
ENCODE_CASES = []
for si, s in enumerate(ENCODE_STRINGS):
    ENCODE_CASES.append((f"gpt2_str{si}_nospecial", "gpt2", None, {"kind": "string", "text": s}))
    ENCODE_CASES.append((f"gpt2_str{si}_eot", "gpt2", [EOT], {"kind": "string", "text": s}))
    ENCODE_CASES.append((f"gpt2_str{si}_overlap", "gpt2", [EOT, EOT + EOT],
                         {"kind": "string", "text": s}))
ENCODE_CASES += [
    ("gpt2_missing_special", "gpt2", ["<|fim|>", EOT, "<|padding|>"],
     {"kind": "string", "text": "a<|fim|>b<|padding|> c <|endoftext|><|padding|><|pad|>"}),
    ("gpt2_address", "gpt2", None, fixture("address.txt")),
    ("gpt2_german", "gpt2", None, fixture("german.txt")),
    ("gpt2_tiny_eot", "gpt2", [EOT], fixture("tinystories_sample.txt")),
    ("gpt2_corpus_en", "gpt2", [EOT], fixture("corpus.en")),
    ("gpt2_synth_mixed_50k", "gpt2", [EOT], synth_spec(1, 50_000, "mixed")),
    ("gpt2_synth_space_20k", "gpt2", [EOT], synth_spec(3, 20_000, "space")),
    ("trained500_corpus_en", "train:corpus_en_500", [EOT], fixture("corpus.en")),
    ("trained500_tiny", "train:corpus_en_500", [EOT], fixture("tinystories_sample.txt")),
    ("trained500_synth_mixed", "train:corpus_en_500", [EOT], synth_spec(1, 50_000, "mixed")),
    ("trained1200_tiny", "train:tiny_1200", [EOT], fixture("tinystories_sample.txt")),
    ("trained3000_tiny", "train:tiny_3000", [EOT], fixture("tinystories_sample.txt")),
    ("trained_mixed_synth", "train:synth_mixed_200k", [EOT], synth_spec(5, 60_000, "mixed")),
]


# ---------------------------------------------------------------------------------------
def hexb(b: bytes) -> str:
    return b.hex()


def import_reference():
    sys.path.insert(0, str(REF))
    logging.disable(logging.CRITICAL)
    from models.tokenizer import train as ref_train  # noqa: E402
    from models.tokenizer.tokenizer import Tokenizer as RefTokenizer  # noqa: E402
    return ref_train, RefTokenizer


def write_json(path: pathlib.Path, obj):
    path.write_text(json.dumps(obj, separators=(",", ":")) + "\n")


def spec_with_digest(spec):
    spec = dict(spec)
    if spec["kind"] == "synth":
        spec["sha256"] = synth_text.sha256_text(input_text(spec))
    return spec


def run_train(ref_train, name, spec, vocab_size, specials, outdir):
    data = input_bytes(spec)
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "input.txt")
        with open(p, "wb") as f:
            f.write(data)
        t0 = time.time()
        with contextlib.redirect_stderr(io.StringIO()):
            vocab, merges = ref_train.train_bpe(p, vocab_size, list(specials))
        dt = time.time() - t0
    obj = {
        "case": name, "input": spec_with_digest(spec), "vocab_size": vocab_size,
        "special_tokens": specials, "reference_seconds": round(dt, 3),
        "merges": [[hexb(a), hexb(b)] for a, b in merges],
        "vocab": [[i, hexb(v)] for i, v in vocab.items()],
    }
    write_json(outdir / f"train_{name}.json", obj)
    print(f"train {name}: {len(merges)} merges in {dt:.2f}s", flush=True)


def run_words(ref_train, name, spec, specials, outdir):
    import regex
    data = input_bytes(spec)
    # the pattern object the reference builds at train.py:143-146
    pat = regex.compile(
        r"""'(?:[sdmt]|ll|ve|re)| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+""",
        regex.UNICODE)
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "input.txt")
        with open(p, "wb") as f:
            f.write(data)
        freq = ref_train.extract_subword_frequencies(p, set(specials), pat)
    rows = sorted((w.encode("utf-8"), c) for w, c in freq.items())
    obj = {"case": name, "input": spec_with_digest(spec), "special_tokens": specials,
           "words": [[hexb(w), c] for w, c in rows]}
    write_json(outdir / f"words_{name}.json", obj)
    print(f"words {name}: {len(rows)} unique", flush=True)


def load_train_golden(outdir, name):
    obj = json.loads((outdir / f"train_{name}.json").read_text())
    vocab = {i: bytes.fromhex(h) for i, h in obj["vocab"]}
    merges = [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in obj["merges"]]
    return vocab, merges


def run_encode(RefTokenizer, name, tok_spec, specials, text_spec, outdir):
    if tok_spec == "gpt2":
        vocab, merges = gpt2_files.load_gpt2(specials)
    else:
        vocab, merges = load_train_golden(outdir, tok_spec.split(":", 1)[1])
    if text_spec["kind"] == "string":
        text = text_spec["text"]
        spec = {"kind": "string", "text_hex": text.encode("utf-8").hex()}
    else:
        text = input_text(text_spec)
        spec = spec_with_digest(text_spec)
    tok = RefTokenizer(dict(vocab), list(merges), None if specials is None else list(specials))
    t0 = time.time()
    ids = tok.encode(text)
    dt = time.time() - t0
    obj = {"case": name, "tokenizer": tok_spec, "special_tokens": specials, "text": spec,
           "reference_seconds": round(dt, 3), "ids": ids}
    write_json(outdir / f"encode_{name}.json", obj)
    print(f"encode {name}: {len(ids)} ids in {dt:.2f}s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    args = ap.parse_args()
    outdir = HERE
    ref_train, RefTokenizer = import_reference()
    want = (lambda n: args.only is None or n in args.only)
    for name, spec, vs, sp in TRAIN_CASES:
        if want(name):
            run_train(ref_train, name, spec, vs, sp, outdir)
    for name, spec, sp in WORD_CASES:
        if want("words_" + name):
            run_words(ref_train, name, spec, sp, outdir)
    for name, tok_spec, sp, tspec in ENCODE_CASES:
        if want("encode_" + name):
            run_encode(RefTokenizer, name, tok_spec, sp, tspec, outdir)
    # the one error case the reference raises on a path argument
    if want("train_bad_utf8"):
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "bad.txt")
            with open(p, "wb") as f:
                f.write(b"valid start \xff\xfe bad bytes")
            try:
                with contextlib.redirect_stderr(io.StringIO()):
                    ref_train.train_bpe(p, 300, [])
                err = None
            except Exception as e:  # noqa: BLE001
                err = type(e).__name__
        write_json(outdir / "error_train_bad_utf8.json",
                   {"case": "bad_utf8", "input_hex": b"valid start \xff\xfe bad bytes".hex(),
                    "vocab_size": 300, "special_tokens": [], "error": err})
        print("bad utf8 ->", err)


if __name__ == "__main__":
    main()
