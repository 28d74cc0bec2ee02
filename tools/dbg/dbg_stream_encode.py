"""Repeat the 1-workgroup streaming encode case and report mismatches (debug driver)."""
import os
import sys
sys.path[:0] = ['tests/golden', 'tests', 'transformer-lm_amd', '.']


def main():
    import gpt2_files
    import synth_text
    import bpe_amd
    import test_gpu_chunks as C
    from oracle import oracle
    os.environ["BPE355_STREAM_WG"] = sys.argv[1] if len(sys.argv) > 1 else "1"
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    text = synth_text.generate(42, 2_500_000, "mixed") + C._boundary_text(4).decode("utf-8")
    want = oracle.encode(vocab, merges, ["<|endoftext|>"], text)
    fails = 0
    for rep in range(12):
        tok = bpe_amd.Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
        try:
            got = tok.encode(text)
        except RuntimeError as e:
            fails += 1
            print(rep, "error", e, flush=True)
            continue
        if got != want:
            fails += 1
            bad = [i for i, (x, y) in enumerate(zip(got, want)) if x != y]
            print(rep, "mismatch", len(got), len(want), bad[:5], flush=True)
    print("fails", fails, "of 12", flush=True)


if __name__ == "__main__":
    main()
