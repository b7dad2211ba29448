"""airspace CLI, the parts that need no GPU: option
handling (reference test/cli_basic_test.py), the console checks of
test/cli_compression_test.py, and the --params grammar, driven through
lib/libairscli.so with the cases of the reference's test/test_params_parse.c."""
import ctypes
import os
import subprocess

import pytest

from conftest import PKG_DIR, load_pkg

CLI = os.path.join(PKG_DIR, "bin", "airspace")
CLI_LIB = os.path.join(PKG_DIR, "lib", "libairscli.so")
VERSION = "0.6.0"  # include/cmp.h CMP_VERSION_STRING (reference lib/cmp.h)
api = load_pkg().cmpapi

OK, EMPTY, MISSING_EQUAL, INVALID_KEY, INVALID_VALUE = range(5)


@pytest.fixture(scope="module")
def cli():
    if not os.path.exists(CLI) or not os.path.exists(CLI_LIB):
        subprocess.run(["make", "-s", "-C", PKG_DIR, "bin/airspace", "lib/libairscli.so"], check=True)

    def run(args, stdin=b""):
        return subprocess.run([CLI] + [str(a) for a in args], input=stdin, capture_output=True, timeout=60)
    return run


@pytest.fixture(scope="module")
def parser(cli):
    lib = ctypes.CDLL(CLI_LIB)
    lib.cmp_params_parse.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    lib.cmp_params_parse.restype = ctypes.c_int
    lib.cmp_params_to_string.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
    lib.cmp_params_to_string.restype = ctypes.c_size_t

    def parse(s, par=None):
        par = par if par is not None else poisoned()
        st = lib.cmp_params_parse(None if s is None else s.encode(), ctypes.byref(par))
        return st, par

    def to_string(par):
        n = lib.cmp_params_to_string(None, 0, ctypes.byref(par))
        buf = ctypes.create_string_buffer(n + 1)
        assert lib.cmp_params_to_string(buf, n + 1, ctypes.byref(par)) == n
        return buf.value.decode()
    return parse, to_string


def poisoned():
    par = api.CmpParams()
    ctypes.memset(ctypes.byref(par), 0xFF, ctypes.sizeof(par))
    return par


def raw(par):
    return bytes(par)


# ---- options (cli_basic_test.py) -------------------------------------------
@pytest.mark.parametrize("args", [["-V"], ["--version"], ["-qvV"]])
def test_version(cli, args):
    r = cli(args)
    assert r.returncode == 0 and VERSION in r.stdout.decode()


@pytest.mark.parametrize("args", [["-qV"], ["--quiet", "--version"], ["-q", "-V"]])
def test_version_minimal(cli, args):
    r = cli(args)
    assert r.returncode == 0 and r.stdout == (VERSION + "\n").encode()


@pytest.mark.parametrize("args", [["-h"], ["--help"]])
def test_help(cli, args):
    r = cli(args)
    assert r.returncode == 0 and b"Usage: " in r.stdout


def test_invalid_long_option(cli):
    r = cli(["--my_invalid_option"])
    assert r.returncode == 1 and b"my_invalid_option" in r.stderr


def test_invalid_short_option(cli):
    r = cli(["-u"])
    assert r.returncode == 1 and b"u" in r.stderr


def test_o_needs_argument(cli):
    r = cli(["-c", "-o"], stdin=bytes.fromhex("0001 0002"))
    assert r.returncode == 1 and b"requires an argument" in r.stderr


@pytest.mark.parametrize("arg", [["-"], []])
def test_abort_stdin_console(cli, arg):
    r = cli(arg + ["-c", "--debug-stdin-is-consol"], stdin=bytes.fromhex("0001 0002"))
    assert r.returncode == 1 and b"stdin" in r.stderr


@pytest.mark.parametrize("arg", [["-"], []])
def test_abort_stdout_console(cli, arg):
    r = cli(arg + ["-c", "--debug-stdout-is-consol"], stdin=bytes.fromhex("0001 0002"))
    assert r.returncode == 1 and b"stdout" in r.stderr


def test_bad_params_option(cli):
    r = cli(["-c", "--params", "primary_preprocessing=DIF", "--stdout"], stdin=bytes.fromhex("0001"))
    assert r.returncode == 1
    assert b"Invalid value 'DIF'" in r.stderr and b"Incorrect parameter option" in r.stderr


def test_quiet_params_error_is_silent(cli):
    r = cli(["-qqq", "-c", "--params=nope=1", "--stdout"], stdin=bytes.fromhex("0001"))
    assert r.returncode == 1 and r.stderr == b""


# ---- the --params grammar (test_params_parse.c) -----------------------------
PRE_CASES = [("NONE", 0), ("DIFF", 1), ("IWT", 2), ("MODEL", 3), ("DiFf", 1), ("PREPROCESS_DIFF", 1),
             ("CMP_PREPROCESS_DIFF", 1), ("CMP_DIFF", 1), ("CmP_pRePrOcEsS_dIfF", 1)]
ENC_CASES = [("UNCOMPRESSED", 0), ("GOLOMB_ZERO", 1), ("GOLOMB_MULTI", 2), ("ENCODER_UNCOMPRESSED", 0),
             ("CMP_ENCODER_UNCOMPRESSED", 0), ("CMP_UNCOMPRESSED", 0), ("CmP_EnCoDeR_uNcOmPrEsSeD", 0)]
BOOL_CASES = [("TRUE", 1), ("FALSE", 0), ("1", 1), ("0", 0), ("CMP_TRUE", 1), ("CMP_FALSE", 0),
              ("Cmp_True", 1), ("Cmp_False", 0)]


def expect(**fields):
    par = poisoned()
    for k, v in fields.items():
        setattr(par, k, v)
    return raw(par)


@pytest.mark.parametrize("key", ["primary_preprocessing", "secondary_preprocessing"])
@pytest.mark.parametrize("name,value", PRE_CASES)
def test_parse_preprocessing(parser, key, name, value):
    st, par = parser[0](f"{key}={name}")
    assert st == OK and raw(par) == expect(**{key: value})


@pytest.mark.parametrize("key", ["primary_encoder_type", "secondary_encoder_type"])
@pytest.mark.parametrize("name,value", ENC_CASES)
def test_parse_encoder(parser, key, name, value):
    st, par = parser[0](f"{key}={name}")
    assert st == OK and raw(par) == expect(**{key: value})


@pytest.mark.parametrize("key", ["checksum_enabled", "uncompressed_fallback_enabled"])
@pytest.mark.parametrize("name,value", BOOL_CASES)
def test_parse_bool(parser, key, name, value):
    st, par = parser[0](f"{key}={name}")
    assert st == OK and raw(par) == expect(**{key: value})


@pytest.mark.parametrize("s,value", [("primary_encoder_param=0", 0), ("primary_encoder_param=42", 42),
                                     ("primary_encoder_param=4294967295", 4294967295),
                                     ("primary_encoder_param=1,primary_encoder_param=42", 42),
                                     ("PrImArY_EnCoDeR_PaRaM=42", 42)])
def test_parse_numbers(parser, s, value):
    st, par = parser[0](s)
    assert st == OK and raw(par) == expect(primary_encoder_param=value)


@pytest.mark.parametrize("s", ["primary_preprocessing=MODEL,", " primary_preprocessing = MODEL , ",
                               "\tprimary_preprocessing\n=\rMODEL\v,\f", ",,primary_preprocessing=MODEL,,"])
def test_parse_separators_and_whitespace(parser, s):
    st, par = parser[0](s)
    assert st == OK and raw(par) == expect(primary_preprocessing=3)


def test_parse_all_parameters(parser):
    s = ("primary_preprocessing = IWT,primary_encoder_type = GOLOMB_MULTI,primary_encoder_param = 12,"
         "primary_encoder_outlier = 0,secondary_iterations = 4294967295,secondary_preprocessing = DIFF,"
         "secondary_encoder_type = GOLOMB_ZERO,secondary_encoder_param = 42,secondary_encoder_outlier = 1,"
         "model_rate = 16,checksum_enabled = FALSE,uncompressed_fallback_enabled = TRUE,")
    st, par = parser[0](s)
    assert st == OK
    assert raw(par) == expect(primary_preprocessing=2, primary_encoder_type=2, primary_encoder_param=12,
                              primary_encoder_outlier=0, secondary_iterations=4294967295,
                              secondary_preprocessing=1, secondary_encoder_type=1, secondary_encoder_param=42,
                              secondary_encoder_outlier=1, model_rate=16, checksum_enabled=0,
                              uncompressed_fallback_enabled=1)


@pytest.mark.parametrize("s", ["", " ", "\t", "\r", "\n", ",", ", ,", None])
def test_detect_empty(parser, s):
    st, par = parser[0](s)
    assert st == EMPTY and raw(par) == raw(poisoned())


@pytest.mark.parametrize("s", ["primary_preprocessing CMP_PREPROCESS_MODEL",
                               "primary_preprocessing CMP_PREPROCESS_MODEL,",
                               "primary_preprocessingCMP_PREPROCESS_MODEL"])
def test_detect_missing_equal(parser, s):
    assert parser[0](s)[0] == MISSING_EQUAL


@pytest.mark.parametrize("v", ["4294967296", "02", "000000000002", "2.2", "2.", ".2", "2 2", "-2", "0x2", "a", ""])
def test_detect_invalid_numbers(parser, v):
    assert parser[0](f"primary_encoder_param={v}")[0] == INVALID_VALUE


@pytest.mark.parametrize("v", ["", ",", "1", "DIF", "=DIFF", "DIF F"])
def test_detect_invalid_enum_names(parser, v):
    assert parser[0](f"primary_preprocessing={v}")[0] == INVALID_VALUE


@pytest.mark.parametrize("s", ["INVALID=3", "=3"])
def test_detect_invalid_keys(parser, s):
    assert parser[0](s)[0] == INVALID_KEY


def test_to_string_all_fields(parser):
    par = api.CmpParams(primary_encoder_type=2, primary_encoder_param=12, secondary_iterations=4294967295,
                        secondary_preprocessing=1, secondary_encoder_type=1, secondary_encoder_param=42,
                        secondary_encoder_outlier=1, model_rate=16, checksum_enabled=0,
                        uncompressed_fallback_enabled=1)
    ctypes.c_int32.from_buffer(par, api.CmpParams.primary_preprocessing.offset).value = -1
    s = parser[1](par)
    for line in ["primary_preprocessing = INVALID,", "primary_encoder_type = GOLOMB_MULTI,",
                 "primary_encoder_param = 12,", "primary_encoder_outlier = 0,",
                 "secondary_iterations = 4294967295,", "secondary_preprocessing = DIFF,",
                 "secondary_encoder_type = GOLOMB_ZERO,", "secondary_encoder_param = 42,",
                 "secondary_encoder_outlier = 1,", "model_rate = 16,", "checksum_enabled = FALSE,",
                 "uncompressed_fallback_enabled = TRUE\n"]:
        assert line in s, (line, s)
    assert s.count(",\n") == 11 and s.endswith("TRUE\n")


def test_to_string_normalises_bools(parser):
    par = api.CmpParams(checksum_enabled=42)
    assert "checksum_enabled = TRUE" in parser[1](par)


def test_to_string_parse_roundtrip(parser):
    par = api.CmpParams(primary_preprocessing=0, primary_encoder_type=2, primary_encoder_param=7,
                        primary_encoder_outlier=99, secondary_iterations=3, secondary_preprocessing=3,
                        secondary_encoder_type=1, secondary_encoder_param=8, secondary_encoder_outlier=5,
                        model_rate=11, checksum_enabled=1, uncompressed_fallback_enabled=0)
    st, back = parser[0](parser[1](par), api.CmpParams())
    assert st == OK and raw(back) == raw(par)


def test_decompress_rejects_broken_frames(cli, tmp_path):
    """The frame walk (24-bit sizes in each header) runs before any GPU work."""
    bad = tmp_path / "bad.air"
    bad.write_bytes(b"\x80\x01\x00\x00\x40" + b"\0" * 20)  # size 64 > file
    r = cli([bad])
    assert r.returncode == 1 and b"not a valid AIRSPACE frame at byte 0" in r.stderr
    short = tmp_path / "short.air"
    short.write_bytes(b"\x80\x01\x00\x00\x10" + b"\0" * 11 + b"\x80")  # one whole 16-byte frame + 1 byte
    r = cli([short])
    assert r.returncode == 1 and b"at byte 16" in r.stderr
