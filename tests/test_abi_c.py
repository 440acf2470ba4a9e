"""The C ABI from a plain C99 client (tests/c/abi_client.c), compiled with gcc
against include/spai.h and linked to libspai.so -- what a Rust/Go/JNI binding
does.  CPU: it compiles with -Wall -Werror as C, links, and the host-only entry
points answer.  GPU: a Connect4 search through the same client equals the
oracle's visit counts (hash evaluator, bit-exact)."""
import os
import subprocess

import pytest

from conftest import REPO

LIBDIR = os.path.join(REPO, "self-play-ai_amd")


@pytest.fixture(scope="module")
def client(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("abi") / "abi_client")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "c", "abi_client.c"), "-L", LIBDIR, "-lspai",
                    "-Wl,-rpath," + LIBDIR, "-o", exe], check=True)
    return exe


def test_c_client_host_entry_points(client):
    out = subprocess.run([client, "host"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    lines = dict(l.split(" ", 1) for l in out.stdout.strip().splitlines())
    assert lines["version"].startswith("spai")
    assert lines["best_action"] == "2"        # last of the equal maxima
    assert lines["sample"] == "2"             # running totals 0.1, 0.6, 1.1 <= 0.65
    assert "empty policy" in lines["empty_error"]


@pytest.mark.gpu
def test_c_client_search_matches_oracle(client, oracle):
    out = subprocess.run([client, "gpu", "64"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    rows = [l.split() for l in out.stdout.splitlines() if l.startswith("tree ")]
    _, _, _, vis, nc = oracle.search_c4([oracle.C4() for _ in range(3)], 64)
    for t, r in enumerate(rows):
        n = int(r[3])
        assert n == nc[t]
        assert [int(v) for v in r[5:5 + n]] == [int(v) for v in vis[t, :n]]
