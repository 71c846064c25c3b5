"""Host emulation of the device codec against the oracle (one lane; one quad for 4D).

The device headers (zfp-par_amd/csrc/hip/{codec_dev,block3}.h) are compiled
with g++ behind a stub hip_runtime.h (tests/emu/stub) in which a wave is one
lane.  This checks the per-lane logic of every encode/decode path -- closed-form
plane coder, fast-path decoder, casts, headers, all modes, f32/f64 -- on the
CPU, bit for bit against the C oracle.  Wave-level behaviour (ballots across
lanes, LDS sharing, copy-out) is covered by the -m gpu tests.
"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(REPO, "tests", "emu")
HIP = os.path.join(REPO, "zfp-par_amd", "csrc", "hip")


def _build(tmp, src, extra=()):
    exe = os.path.join(tmp, os.path.splitext(os.path.basename(src))[0])
    cmd = ["g++", "-O2", "-std=c++17", "-I" + os.path.join(EMU, "stub"), "-I" + HIP, "-o", exe,
           os.path.join(EMU, src), *extra, "-lm"]
    subprocess.check_call(cmd)
    return exe


@pytest.fixture(scope="module")
def oracle_obj(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("emu"))
    obj = os.path.join(d, "zfp_oracle.o")
    subprocess.check_call(["gcc", "-O2", "-c", "-I" + os.path.join(REPO, "oracle"), "-o", obj,
                           os.path.join(REPO, "oracle", "zfp_oracle.c")])
    return d, obj


def test_plane_decoder_fast_path_matches_reference_loop(oracle_obj):
    d, _ = oracle_obj
    r = subprocess.run([_build(d, "dec_emu.cpp")], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


def test_block_codec_matches_oracle_all_modes(oracle_obj):
    d, obj = oracle_obj
    r = subprocess.run([_build(d, "block_emu.cpp", [obj])], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(" 0/3000 bad") == 32, r.stdout


def test_plane_decoder_dense_switch_matches_reference_loop(tmp_path):
    """decode_planes32 leaving its 32-bit body after any slow plane (the switch a wave
    takes after a dense plane), against the same reference streams."""
    exe = os.path.join(str(tmp_path), "plane_emu_dense")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-DZFP_DEC32_DENSE=0", "-I" + os.path.join(EMU, "stub"),
                           "-I" + HIP, "-o", exe, os.path.join(EMU, "plane_emu.cpp"), "-lm"])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr


def test_plane_coder_matches_reference_loop(tmp_path):
    """code_planes vs a literal restatement of encode.c:92-132 on adversarial planes."""
    r = subprocess.run([_build(str(tmp_path), "plane_emu.cpp")], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


def test_4d_quad_codec_matches_oracle_all_modes(oracle_obj):
    """block4.h run as four threads (one quad): DPP permutes and barriers are a
    four-thread rendezvous, so the quad reductions, the w-lift exchange and the
    segment-parallel plane coder/decoder are checked bit for bit on the CPU."""
    d, obj = oracle_obj
    r = subprocess.run([_build(d, "quad_emu.cpp", [obj, "-pthread"])], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(" 0/200 bad") == 32, r.stdout


def test_index_scan_matches_oracle_block_starts(oracle_obj):
    """scan.h (index-free variable-rate decode): per-block bit lengths and the
    resynchronising segment passes recover every block start of oracle streams
    in precision, accuracy, reversible and expert modes, 3D and 4D, f32 and f64,
    at several segment sizes and unaligned stream offsets."""
    d, obj = oracle_obj
    r = subprocess.run([_build(d, "scan_emu.cpp", [obj, "-DZFP_SCAN_RING_WORDS=4"])], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "scan mismatches 0" in r.stdout, r.stdout
