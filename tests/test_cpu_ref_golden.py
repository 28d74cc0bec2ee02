"""Pin oracle/cpu_ref.py -- the pure-Python restatement of the reference trainer that bench.py
times as `cpu_baseline` -- against every train golden produced by the reference itself
(tests/golden/train_*.json, make_golden.py).  CPU only."""
import pytest

import golden_cases as G
from oracle import cpu_ref
from oracle import oracle


@pytest.mark.parametrize("name", G.names("train"))
def test_cpu_ref_train_matches_reference(name):
    o, vocab, merges = G.train_expect(name)
    data = G.input_bytes(o["input"])
    text = oracle.decode_text(data).decode("utf-8")   # the reference's text-mode read
    got_vocab, got_merges, info = cpu_ref.train(text, o["vocab_size"], o["special_tokens"])
    assert info["complete"]
    assert got_merges == merges
    assert got_vocab == vocab


@pytest.mark.parametrize("name", G.names("encode"))
def test_cpu_ref_encode_matches_reference(name):
    """the encode port bench.py times (cpu_baseline.encode) against every encode golden"""
    o = G.load("encode", name)
    vocab, merges = G.tokenizer_inputs(o)
    enc = cpu_ref.Encoder(vocab, merges, o["special_tokens"])
    assert enc.encode(G.encode_text(o)) == o["ids"]


def test_cpu_baseline_growth_curve():
    """the CPU baseline's extrapolation model (oracle/cpu_port_growth.json, from a complete run of
    the port on the 16 MB bench sample): the whole run's mean round is dearer than the first
    rounds' mean, and a complete run needs no correction"""
    import json
    import pathlib
    from oracle import cpu_bench
    g = json.loads((pathlib.Path(cpu_bench.__file__).parent / "cpu_port_growth.json").read_text())
    pts = g["points"]
    assert pts[-1][0] == g["rounds_total"] == 31743
    assert all(b[0] > a[0] and b[1] >= a[1] for a, b in zip(pts, pts[1:]))   # cumulative
    n, v = g["bytes"], g["vocab"]
    f, ok = cpu_bench.growth_factor(g["rounds_total"], g["rounds_total"], n, v)
    assert ok and abs(f - 1.0) < 1e-9
    for r in (10, 199, 450, 1240, 5000):
        f, ok = cpu_bench.growth_factor(r, g["rounds_total"], n, v)
        assert ok and f > 1.5
    # the curve is validated only on the sample it was measured on
    assert cpu_bench.growth_factor(450, g["rounds_total"], 4 * n, v)[1] is False
    assert cpu_bench.growth_factor(450, g["rounds_total"], n, 10000)[1] is False
    # the flat rate of the first rounds under-estimated the complete run by ~86 %
    assert g["flat_projection_error"] < -0.5
