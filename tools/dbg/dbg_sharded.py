"""Debug driver: run the 2-rank host-comm sharded trainer on a synth_text corpus with tracing,
and compare with the single-process oracle."""
import os
import sys
import time

sys.path[:0] = ['tests', 'transformer-lm_amd', '.']


def main():
    os.environ['BPE355_TRACE'] = '1'
    import test_gpu_sharded as T
    import synth_text
    from oracle import oracle
    import bpe_amd
    t0 = time.time()
    data = synth_text.generate(31, int(sys.argv[1]), "ascii").encode("utf-8")
    vs = int(sys.argv[2])
    want = oracle.train_raw(data, vs, ["<|endoftext|>"])
    single = bpe_amd.train_bpe_bytes(data, vs, ["<|endoftext|>"])
    print('gen+oracle', time.time() - t0, 'single==oracle', single == want, flush=True)
    out = T.run_sharded(data, 2, vs, ["<|endoftext|>"])
    for r, v in out.items():
        if isinstance(v, str):
            print('rank', r, 'error', v)
            continue
        m = v[1]
        first = next((i for i, (x, y) in enumerate(zip(m, want[1])) if x != y), None)
        print('rank', r, len(m), 'first mismatch', first, m[first] if first is not None else '',
              want[1][first] if first is not None else '', flush=True)


if __name__ == '__main__':
    main()
