"""airspace CLI on the GPU: the reference's
test/cli_compression_test.py cases, frames checked byte for byte against the
CPU oracle fed the same files through one context (header identifiers
excepted: they come from the clock), and .air files decompressed back to the
input samples.

Every compression case runs twice: on this build's airspace
(airs-compression_amd/bin/airspace) and on the REFERENCE's own command-line
tool, programs/airspacecli.c with its helpers compiled unchanged from the
reference tree and linked to libairscmp.so only (tests/dropin/Makefile; built
by __graft_entry__.build() where the reference is present): the literal
drop-in of north_star ("drops in under programs/airspacecli").  The
reference tool has no decompression (programs/airspacecli.c:421-423), so the
round trips decode its .air output with this build's airspace."""
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG_DIR, ROOT, load_pkg

pytestmark = pytest.mark.gpu
CLI = os.path.join(PKG_DIR, "bin", "airspace")
REF_CLI = os.path.join(ROOT, "tests", "dropin", "airspacecli")
api = load_pkg().cmpapi
DATA1 = bytes.fromhex("0001 0002")
DATA2 = bytes.fromhex("0003 0004")
HDR = 16  # NONE + UNCOMPRESSED header (the CLI's default parameters)


@pytest.fixture(params=["airspace", "reference"])
def cli(request):
    """The compressing tool under test: this build's CLI, or the reference's
    airspacecli linked to libairscmp.so."""
    if request.param == "airspace":
        return CLI
    if not os.path.exists(REF_CLI):
        pytest.skip("tests/dropin/airspacecli not built (the reference tree was absent at build time)")
    ldd = subprocess.run(["ldd", REF_CLI], capture_output=True, text=True).stdout
    assert "libairscmp.so" in ldd, ldd  # the reference tool runs on this library
    return REF_CLI


def run(args, cwd, stdin=b"", tool=CLI):
    return subprocess.run([tool] + [str(a) for a in args], input=stdin, capture_output=True, cwd=cwd, timeout=120)


@pytest.fixture
def files(tmp_path, prod):
    if not prod.gpu_available():
        pytest.fail("GPU test run without a usable HIP device")
    f1, f2 = tmp_path / "file_1.bin", tmp_path / "file_2.bin"
    f1.write_bytes(DATA1)
    f2.write_bytes(DATA2)
    return tmp_path, f1, f2


def ok(r):
    assert r.returncode == 0, r.stderr.decode()
    return r


# ---- cli_compression_test.py ------------------------------------------------
def test_two_files_to_dev_null(cli, files):
    d, f1, f2 = files
    r = ok(run(["-c", f1, f2, "-o", os.devnull, "--quiet"], d, tool=cli))
    assert r.stderr == b""


def test_two_files_to_stdout(cli, files):
    d, f1, f2 = files
    r = ok(run(["-c", f1, f2, "--stdout"], d, tool=cli))
    assert r.stderr == b""
    assert r.stdout[HDR:HDR + 4] == DATA1 and r.stdout[2 * HDR + 4:] == DATA2


def test_two_files_normally(cli, files):
    d, f1, f2 = files
    r = ok(run(["-c", f1, f2, "--quiet"], d, tool=cli))
    assert r.stderr == b""
    assert (d / "file_1.bin.air").read_bytes()[HDR:] == DATA1
    assert (d / "file_2.bin.air").read_bytes()[HDR:] == DATA2


@pytest.mark.parametrize("arg", [["-"], []])
def test_stdin_to_stdout(cli, files, arg):
    d, _, _ = files
    r = ok(run(["-c"] + arg, d, stdin=DATA1, tool=cli))
    assert r.stdout[HDR:] == DATA1 and len(r.stdout) == HDR + 4


def test_file_to_output_file(cli, files):
    d, f1, _ = files
    ok(run(["-c", f1, "-o", d / "output.air", "--quiet"], d, tool=cli))
    assert (d / "output.air").read_bytes()[HDR:] == DATA1


def test_file_and_stdin(cli, files):
    d, f1, _ = files
    r = ok(run(["-c", f1, "-", "--quiet"], d, stdin=DATA2, tool=cli))
    assert r.stdout[HDR:HDR + 4] == DATA1 and r.stdout[2 * HDR + 4:] == DATA2


def test_files_of_different_sizes(cli, files):
    d, f1, _ = files
    small = d / "small_file.bin"
    small.write_bytes(bytes.fromhex("0003"))
    ok(run(["-c", f1, small, "--quiet"], d, tool=cli))
    assert (d / "file_1.bin.air").read_bytes()[HDR:] == DATA1
    assert (d / "small_file.bin.air").read_bytes()[HDR:] == bytes.fromhex("0003")


def test_summary_line(cli, files):
    d, f1, f2 = files
    r = ok(run(["-c", f1, f2], d, tool=cli))
    assert r.stderr.startswith(b"2 files compressed: ")
    r = ok(run(["-c", d / "file_1.bin", "-o", d / "one.air"], d, tool=cli))
    assert b"file_1.bin: " in r.stderr and b"one.air" in r.stderr


def test_not_overwrite_existing_file(cli, files):
    d, f1, f2 = files
    existing = d / "existing_file.txt"
    existing.write_text("Do not overwrite this file!")
    r = run(["-c", f1, f2, "-o", existing], d, tool=cli)
    assert r.returncode == 1 and b"already exists" in r.stderr
    assert existing.read_text() == "Do not overwrite this file!"


def test_not_overwrite_existing_directory(cli, files):
    d, f1, f2 = files
    (d / "existing_dir").mkdir()
    r = run(["-c", f1, f2, "-o", d / "existing_dir"], d, tool=cli)
    assert r.returncode == 1 and b"is a directory" in r.stderr


def test_not_overwrite_input_file(cli, files):
    d, f1, _ = files
    r = run(["-c", f1, "-o", f1], d, tool=cli)
    assert r.returncode == 1 and b"already exists" in r.stderr and f1.read_bytes() == DATA1


def test_odd_sized_and_empty_files(cli, files):
    d, f1, _ = files
    odd, empty = d / "odd.bin", d / "empty.bin"
    odd.write_bytes(b"\x00\x01\x02")
    empty.write_bytes(b"")
    r = run(["-c", f1, odd, "--quiet"], d, tool=cli)
    assert r.returncode == 1 and b"multiple of 2" in r.stderr
    assert (d / "file_1.bin.air").read_bytes()[HDR:] == DATA1  # files before the bad one are written
    r = run(["-c", empty], d, tool=cli)
    assert r.returncode == 1 and b"is empty" in r.stderr


# ---- frames vs the oracle, and decompression --------------------------------
PARAMS = {
    "diff_zero32": dict(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=32),
    "multi_ck": dict(primary_preprocessing=1, primary_encoder_type=2, primary_encoder_param=10,
                     primary_encoder_outlier=300, checksum_enabled=1),
    "model_chain": dict(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=16,
                        secondary_iterations=3, secondary_preprocessing=3, secondary_encoder_type=1,
                        secondary_encoder_param=8, model_rate=11),
    "iwt": dict(primary_preprocessing=2, primary_encoder_type=2, primary_encoder_param=12,
                primary_encoder_outlier=100),
    "fallback": dict(primary_preprocessing=0, primary_encoder_type=1, primary_encoder_param=1,
                     uncompressed_fallback_enabled=1),
    # IWT primaries, MODEL secondaries and the fallback: the device work buffer
    # carries the model through the batch (round 5: these sets batch too)
    "iwt_model_fb": dict(primary_preprocessing=2, primary_encoder_type=1, primary_encoder_param=16,
                         secondary_iterations=2, secondary_preprocessing=3, secondary_encoder_type=1,
                         secondary_encoder_param=8, model_rate=7, uncompressed_fallback_enabled=1,
                         checksum_enabled=1),
}


def params_arg(p):
    names = {"primary_preprocessing": ["NONE", "DIFF", "IWT", "MODEL"],
             "secondary_preprocessing": ["NONE", "DIFF", "IWT", "MODEL"],
             "primary_encoder_type": ["UNCOMPRESSED", "GOLOMB_ZERO", "GOLOMB_MULTI"],
             "secondary_encoder_type": ["UNCOMPRESSED", "GOLOMB_ZERO", "GOLOMB_MULTI"]}
    return ",".join(f"{k}={names[k][v] if k in names else v}" for k, v in p.items())


def sample_files(d, kind, rng):
    """Seven files: four of 5000 samples, two of 777, one of 5000 (runs of equal
    size, so the batched path splits), or all 3000 for parameter sets with a
    work buffer."""
    sizes = [3000] * 6 if kind in ("model_chain", "iwt", "iwt_model_fb") else [5000, 5000, 5000, 5000, 777, 777, 5000]
    base = np.cumsum(rng.integers(-200, 200, max(sizes)))
    paths, xs = [], []
    for i, n in enumerate(sizes):
        if kind == "fallback":
            x = rng.integers(0, 65536, n).astype(np.uint16)
        else:
            x = ((base[:n] + rng.integers(-30, 30, n) + 1000 * i) & 0xFFFF).astype(np.uint16)
        p = d / f"s{i}.dat"
        p.write_bytes(x.astype(">u2").tobytes())
        paths.append(p)
        xs.append(x)
    return paths, xs


def split_frames(blob):
    out, pos = [], 0
    while pos < len(blob):
        size = int.from_bytes(blob[pos + 2:pos + 5], "big")
        assert size >= 16
        out.append(blob[pos:pos + size])
        pos += size
    return out


def masked(frame):
    return frame[:8] + b"\0" * 6 + frame[14:]  # identifier bytes 8-13 come from the clock


@pytest.mark.parametrize("kind", list(PARAMS))
def test_frames_match_oracle_and_decompress(tmp_path, prod, orc, kind, cli):
    if not prod.gpu_available():
        pytest.fail("GPU test run without a usable HIP device")
    rng = np.random.default_rng(sum(map(ord, kind)))
    paths, xs = sample_files(tmp_path, kind, rng)
    r = ok(run(["-c", "--params", params_arg(PARAMS[kind])] + paths + ["--stdout"], tmp_path, tool=cli))
    frames = split_frames(r.stdout)
    assert len(frames) == len(xs)

    par = api.CmpParams(**PARAMS[kind])
    ctx = api.CmpContext()
    wbs = orc.cal_work_buf_size(par, 2 * len(xs[0]))
    if wbs:
        wb = api.aligned_empty(wbs, fill=0)
        assert not api.is_error(orc.initialise(ctx, par, wb, wbs))
    else:
        assert not api.is_error(orc.initialise(ctx, par))
    for i, x in enumerate(xs):
        cap = 26 + 6 * len(x) + 64
        dst = api.aligned_empty(cap)
        got = orc.compress_u16(ctx, dst, cap, x)
        assert not api.is_error(got), api.error_name(got)
        assert masked(frames[i]) == masked(bytes(dst[:got])), (kind, i)

    # the concatenated frames decompress back to the concatenated samples
    (tmp_path / "all.air").write_bytes(r.stdout)
    ok(run(["-q", tmp_path / "all.air"], tmp_path))
    want = b"".join(x.astype(">u2").tobytes() for x in xs)
    assert (tmp_path / "all").read_bytes() == want


def test_decompress_errors(files):
    d, f1, _ = files
    ok(run(["-c", f1, "--quiet"], d))
    r = run(["-q", d / "file_1.bin.air"], d)  # would write file_1.bin, which exists
    assert r.returncode == 1 and b"already exists" in r.stderr
    (d / "x.bin").write_bytes((d / "file_1.bin.air").read_bytes())
    r = run([d / "x.bin"], d)
    assert r.returncode == 1 and b"unknown suffix" in r.stderr
    (d / "bad.air").write_bytes(b"\x80\x01\x00\x00\x40" + b"\0" * 20)
    r = run([d / "bad.air"], d)
    assert r.returncode == 1 and b"not a valid AIRSPACE frame" in r.stderr
    r = ok(run(["--stdout", d / "file_1.bin.air"], d))
    assert r.stdout == DATA1
