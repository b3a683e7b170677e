"""The R boundary (r_shim/RcppExports.cpp) compiled and driven without R.

tests/r_api/ declares the part of R's C API the shim uses and mock_r.cpp implements it in memory,
with recording stand-ins for libbrr's one-shot entry points.  Checked: integer / logical inputs
are coerced to double as Rcpp's input_parameter<Eigen::MatrixXd> does (src/RcppExports.cpp:14-33,
43-55, 65-80, 90-104); N = epsilon.size() for BRV2Grstart (src/BRv2Grstart.cpp:81) and Y.size()
otherwise (src/BayesRv2.cpp:64); cva is repacked to `groups` rows; size mismatches become R errors
with the PROTECT stack balanced; the four .Call symbols carry the reference arities
(src/RcppExports.cpp:110-121).
"""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(REPO, "r_shim", "RcppExports.cpp")
API = os.path.join(REPO, "tests", "r_api")


def _gxx():
    g = shutil.which("g++")
    if not g:
        pytest.skip("g++ not available")
    return g


@pytest.fixture(scope="module")
def runs(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("rshim") / "mock_r")
    subprocess.run([_gxx(), "-std=c++17", "-Wall", "-Werror", "-Wno-cast-function-type", f"-I{API}",
                    f"-I{REPO}/include", SHIM, os.path.join(API, "mock_r.cpp"), "-o", exe], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    res = {}
    for line in out.strip().splitlines():
        name, rec, err, nprot = line.split("|")
        res[name] = (rec, err, int(nprot))
    return res


def test_shim_compiles_warning_free():
    subprocess.run([_gxx(), "-std=c++17", "-Wall", "-Wextra", "-Werror", "-Wno-cast-function-type",
                    "-fsyntax-only", f"-I{API}", f"-I{REPO}/include", SHIM], check=True)


def test_call_entries_match_reference_arity():
    src = open(SHIM).read()
    ent = dict(re.findall(r'\{"(_BayesRRcpp_\w+)", \(DL_FUNC\)&\w+, (\d+)\}', src))
    assert ent == {"_BayesRRcpp_BRV2Grstart": "20", "_BayesRRcpp_BayesRSamplerV2": "13",
                   "_BayesRRcpp_BayesRSamplerV2Groups": "16", "_BayesRRcpp_HorseshoeR": "15"}


def test_integer_genotypes_coerced(runs):
    rec, err, nprot = runs["v2_int"]
    assert not err and nprot == 0
    assert "N=3 M=2" in rec and "X=[0,1,2,2,1,0]" in rec and "Y=[1,2,3]" in rec
    assert "seed=7 it=20 burn=10 thin=2" in rec and "cva=[0.0001,0.001,0.01]" in rec


def test_logical_matrix_coerced(runs):
    rec, err, nprot = runs["hs_logical_x"]
    assert not err and nprot == 0 and "N=2 M=1" in rec and "X=[1,0]" in rec


def test_restart_takes_n_from_epsilon(runs):
    rec, err, nprot = runs["restart"]
    assert not err and nprot == 0
    assert "N=3 M=2" in rec and "comp=[2,0]" in rec and "beta=[0.5,0]" in rec
    rec, err, nprot = runs["restart_eps_mismatch"]
    assert "epsilon has 2 entries" in err and rec == "" and nprot == 0


def test_groups_cva_repacked(runs):
    rec, err, nprot = runs["groups_cva"]
    assert not err and nprot == 0
    assert "G=2" in rec and "cva=[1,2,10,20]" in rec and "gA=[0,1,1]" in rec and "F=1" in rec
    rec, err, _ = runs["groups_cva_short"]
    assert "fewer than groups" in err and rec == ""


def test_errors_reach_r(runs):
    assert "Y has 2 entries" in runs["v2_rows_mismatch"][1]
    assert "must be numeric" in runs["v2_string_x"][1]
    assert all(v[2] == 0 for v in runs.values())  # PROTECT stack balanced on every path
