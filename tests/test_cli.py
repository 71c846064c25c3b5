"""Command-line tool (zfp-par_amd/bin/zfp), the C1 path of SURVEY §8 (a21).

The reference CLI is utils/zfp.c:139-629: `-f -3 nx ny nz -r 16 -i in -z out`
writes the raw stream (no header) that zfp_compress produces, word-flushed;
`-h` prepends the full header; `-z ... -o ...` decompresses.  GPU tests check
the output bytes against the oracle's stream (and against the reference CLI
built from source in oracle/_ref when it is present).
"""
import os
import subprocess

import numpy as np
import pytest

from pyoracle import REF_CLI, params_precision, params_rate, params_reversible

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "zfp-par_amd", "bin", "zfp")


def run(args, **kw):
    return subprocess.run([CLI] + args, capture_output=True, **kw)


@pytest.fixture(scope="module")
def cli():
    if not os.path.exists(CLI):
        raise RuntimeError("zfp-par_amd/bin/zfp not built (make -C zfp-par_amd)")
    return CLI


# ---- argument handling (no GPU needed: nothing is compressed) ----

def test_no_arguments_prints_usage(cli):
    r = run([])
    assert r.returncode == 1
    assert b"Usage: zfp <options>" in r.stderr


@pytest.mark.parametrize("args,msg", [
    (["-f", "-3", "4", "4", "4", "-r", "8"], b"must specify uncompressed or compressed input file"),
    (["-i", "x.raw", "-3", "4", "4", "4", "-r", "8"], b"must specify scalar type"),
    (["-i", "x.raw", "-f", "-r", "8"], b"must specify array dimensions"),
    (["-i", "x.raw", "-f", "-3", "4", "4", "4"], b"must specify compression parameters"),
    (["-z", "x.zfp", "-h", "-f"], b"cannot specify both field type/size and header"),
    (["-f", "-3", "0", "4", "4", "-r", "8", "-i", "x"], b"array size must be nonzero"),
])
def test_argument_errors(cli, args, msg):
    r = run(args)
    assert r.returncode == 1
    assert msg in r.stderr


@pytest.mark.parametrize("args", [["-q", "extra"], ["-x", "bogus"], ["-t", "f16"], ["-r"]])
def test_bad_options_print_usage(cli, args):
    r = run(args)
    assert r.returncode == 1 and b"Usage" in r.stderr


# ---- compression through the CLI on the GPU ----

def _field(oracle, shape, dtype):
    return oracle.smooth_field(len(shape), dtype, min_total=int(np.prod(shape))).ravel()[: int(np.prod(shape))].reshape(shape)


MODES = [("r", "16", lambda t: params_rate(16, t, 3)), ("p", "20", lambda t: params_precision(20)),
         ("R", None, lambda t: params_reversible())]


@pytest.mark.gpu
@pytest.mark.parametrize("flag,val,params", MODES, ids=[m[0] for m in MODES])
@pytest.mark.parametrize("dtype", [np.float32, np.float64], ids=["f32", "f64"])
def test_cli_stream_matches_oracle(cli, product, oracle, tmp_path, flag, val, params, dtype):
    shape = (20, 33, 40)  # nz, ny, nx
    arr = _field(oracle, shape, dtype)
    raw = tmp_path / "in.raw"
    arr.tofile(raw)
    out = tmp_path / "out.zfp"
    back = tmp_path / "back.raw"
    t = "-f" if dtype == np.float32 else "-d"
    mode = ["-" + flag] + ([val] if val else [])
    r = run([t, "-3", "40", "33", "20"] + mode + ["-i", str(raw), "-z", str(out), "-o", str(back), "-q"])
    assert r.returncode == 0, r.stderr
    ztype = 3 if dtype == np.float32 else 4
    words, end = oracle.compress_words(arr, params(ztype))
    assert out.read_bytes() == words.tobytes()
    want, _ = oracle.decompress_words(words, shape, dtype, params(ztype))
    assert np.array_equal(np.fromfile(back, dtype=dtype).reshape(shape).view(np.uint8), want.view(np.uint8))
    if os.path.exists(REF_CLI):
        ref = tmp_path / "ref.zfp"
        rr = subprocess.run([REF_CLI, t, "-3", "40", "33", "20"] + mode + ["-i", str(raw), "-z", str(ref), "-q"],
                            capture_output=True)
        assert rr.returncode == 0, rr.stderr
        assert out.read_bytes() == ref.read_bytes()


@pytest.mark.gpu
def test_cli_header_round_trip_and_stats(cli, product, oracle, tmp_path):
    shape = (16, 24, 32)
    arr = _field(oracle, shape, np.float32)
    raw = tmp_path / "in.raw"
    arr.tofile(raw)
    z = tmp_path / "h.zfp"
    r = run(["-f", "-3", "32", "24", "16", "-r", "8", "-h", "-i", str(raw), "-z", str(z), "-s"])
    assert r.returncode == 0, r.stderr
    assert b"type=float nx=32 ny=24 nz=16 nw=1" in r.stderr and b"rmse=" in r.stderr
    assert z.read_bytes()[:4] == b"zfp\x05"
    o = tmp_path / "o.raw"
    r = run(["-z", str(z), "-h", "-o", str(o), "-q"])
    assert r.returncode == 0, r.stderr
    words, _ = oracle.compress_words(arr, params_rate(8, 3, 3))
    want, _ = oracle.decompress_words(words, shape, np.float32, params_rate(8, 3, 3))
    assert np.array_equal(np.fromfile(o, dtype=np.float32).reshape(shape), want)
    if os.path.exists(REF_CLI):
        ref = tmp_path / "ref.zfp"
        rr = subprocess.run([REF_CLI, "-f", "-3", "32", "24", "16", "-r", "8", "-h", "-i", str(raw), "-z", str(ref),
                             "-q"], capture_output=True)
        assert rr.returncode == 0 and z.read_bytes() == ref.read_bytes()


@pytest.mark.gpu
@pytest.mark.parametrize("t,dims,mode", [
    ("i32", ["-2", "45", "38"], ["-r", "12"]),
    ("i64", ["-4", "9", "10", "11", "6"], ["-p", "40"]),
    ("f64", ["-1", "1001"], ["-R"]),
    ("f32", ["-2", "64", "33"], ["-a", "1e-3"]),
], ids=["2d-i32-rate", "4d-i64-precision", "1d-f64-reversible", "2d-f32-accuracy"])
def test_cli_other_instantiations_match_reference_cli(cli, product, tmp_path, t, dims, mode):
    """1D/2D and integer fields through bin/zfp on the GPU, against the reference's own CLI."""
    if not os.path.exists(REF_CLI):
        pytest.skip("reference CLI not built (oracle/_ref)")
    dtype = {"i32": np.int32, "i64": np.int64, "f32": np.float32, "f64": np.float64}[t]
    n = int(np.prod([int(x) for x in dims[1:]]))
    rng = np.random.default_rng(3)
    x = np.arange(n, dtype=np.float64)
    vals = 1000 * np.sin(0.01 * x) + rng.standard_normal(n)
    arr = (vals * (1 << 16)).astype(dtype) if np.dtype(dtype).kind == "i" else vals.astype(dtype)
    raw = tmp_path / "in.raw"
    arr.tofile(raw)
    out, back, ref, rback = (tmp_path / f for f in ("out.zfp", "back.raw", "ref.zfp", "rback.raw"))
    r = run(["-t", t] + dims + mode + ["-i", str(raw), "-z", str(out), "-o", str(back), "-q"])
    assert r.returncode == 0, r.stderr
    rr = subprocess.run([REF_CLI, "-t", t] + dims + mode + ["-i", str(raw), "-z", str(ref), "-o", str(rback), "-q"],
                        capture_output=True)
    assert rr.returncode == 0, rr.stderr
    assert out.read_bytes() == ref.read_bytes()
    assert back.read_bytes() == rback.read_bytes()
