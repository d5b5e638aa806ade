"""The host-side file code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU).

csrc/gc_io_host.cpp reads the reference's JSON graphs (graph.py:15-28) and the binary .gcsr
files the drop-in CLI accepts -- untrusted input -- and writes the reference's JSON outputs
(coloring.py:238-241, graph.py:10-12); csrc/gc_gen_host.cpp is the graph.py:30-43 generator.
tests/host_asan/driver.cpp links exactly those sources with -fsanitize=address,undefined (SURVEY
§5: an optional host sanitizer build) and runs them on the golden graphs, on truncated and
corrupted files and on generated graphs; any sanitizer report fails the test (the driver exits
non-zero).  No GPU code is involved.
"""
import json
import os
import random
import shutil
import struct
import subprocess

import numpy as np
import pytest

from conftest import PKG_DIR, REPO, golden_names, load_golden

CSRC = os.path.join(PKG_DIR, "csrc")
ENV = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=1:abort_on_error=0",
           UBSAN_OPTIONS="print_stacktrace=1")


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = str(tmp_path_factory.mktemp("asan") / "gc_host_asan")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-I", os.path.join(REPO, "include"), os.path.join(REPO, "tests", "host_asan", "driver.cpp"),
           os.path.join(CSRC, "gc_io_host.cpp"), os.path.join(CSRC, "gc_gen_host.cpp"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def _run(exe, *args):
    r = subprocess.run([exe, *args], capture_output=True, text=True, env=ENV, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return [line.split() for line in r.stdout.splitlines()]


def _graph_json(rec):
    return json.dumps([{"id": g[0], "neighbors": g[1], "color": -1} for g in rec["graph"]], indent=4)


def test_writers_and_round_trips(driver, tmp_path):
    out = _run(driver, "write", str(tmp_path))
    assert out[0] == ["write", "0"]
    assert all(line[0] == "0" for line in out[1:]) and len(out) == 5
    # the JSON writers are byte-identical to json.dump(indent=4) (checked elsewhere); parse them
    g = json.load(open(tmp_path / "g.json"))
    assert len(g) == 50 and json.load(open(tmp_path / "c0.json")) == []


def test_golden_graphs(driver, tmp_path):
    paths, expect = [], []
    for name in golden_names():
        rec = load_golden(name)
        if not rec.get("graph"):
            continue
        p = tmp_path / f"{name}.json"
        p.write_text(_graph_json(rec))
        paths.append(str(p))
        expect.append(rec)
    res = _run(driver, "read", *paths)
    assert len(res) == len(paths)
    ok = 0
    for (st, n, nnz, _), rec in zip(res, expect):
        st = int(st)
        assert st in (0, -6, -7), st  # read, left to Python's json, or KeyError
        if st == 0:
            ok += 1
            assert int(n) == len(rec["graph"]) and int(nnz) == sum(len(g[1]) for g in rec["graph"])
    assert ok > len(paths) // 2


def test_truncated_and_corrupted_json(driver, tmp_path):
    rng = random.Random(5)
    rec = load_golden("gen_1000_8_s1")
    text = _graph_json(rec).encode()
    paths = []
    cuts = sorted(rng.sample(range(len(text)), 60)) + [0, 1, 2, len(text) - 1]
    for i, c in enumerate(cuts):
        p = tmp_path / f"cut{i}.json"
        p.write_bytes(text[:c])
        paths.append(str(p))
    for i in range(120):
        b = bytearray(text[: rng.randint(1, 4000)] if i % 2 else text)
        for _ in range(rng.randint(1, 8)):
            b[rng.randrange(len(b))] = rng.choice(b'[]{},:"-0123456789 \\\nxe+.\x00\xff')
        p = tmp_path / f"flip{i}.json"
        p.write_bytes(bytes(b))
        paths.append(str(p))
    specials = [b"", b"[]", b"[", b"]", b"[{}]", b"{}", b"[[]]", b'[{"id": 1}]', b'[{"neighbors": []}]',
                b'[{"id": 99999999999999999999, "neighbors": []}]', b'[{"id": -9223372036854775808, "neighbors": []}]',
                b'[{"id": 1, "neighbors": [1, 1, 1]}]', b'[{"id": 1, "neighbors": [2]}]', b"[" * 100000,
                b'[{"id": 1, "neighbors": [' + b"1," * 50000 + b'1]}]', b'[{"id": 1, "neighbors": [], "x": [[[[{}]]]]}]',
                '[{"id": 1, "neighbors": [], "c": "é"}]'.encode(), b'[{"id": 1e3, "neighbors": []}]',
                b'[{"id": 1, "neighbors": []},]', b'[{"id": 1, "neighbors": []}] x']
    for i, b in enumerate(specials):
        p = tmp_path / f"sp{i}.json"
        p.write_bytes(b)
        paths.append(str(p))
    res = _run(driver, "read", *paths)
    assert len(res) == len(paths)
    assert all(int(r[0]) in (0, -6, -7, -8) for r in res)


def test_gcsr_corruptions(driver, tmp_path):
    _run(driver, "write", str(tmp_path))
    good = (tmp_path / "g.gcsr").read_bytes()
    rng = random.Random(9)
    paths = [str(tmp_path / "g.gcsr")]
    variants = [good[:c] for c in (0, 7, 8, 31, 32, 40, len(good) - 1)]
    for field, fmt in ((8, "<q"), (16, "<q"), (24, "<I"), (28, "<I")):
        for val in (-1, 0, 1, 2**31, 2**62, 2**63 - 1) if fmt == "<q" else (0, 1, 2, 2**31):
            b = bytearray(good)
            b[field:field + struct.calcsize(fmt)] = struct.pack(fmt, val)
            variants.append(bytes(b))
    # a crafted header whose 4 * nnz wraps the size arithmetic to the file's true size (row
    # offsets monotone up to nnz, so every later check would pass and read past `col`)
    n = struct.unpack("<q", good[8:16])[0]
    nnz = 2**62
    crafted = bytearray(good[:32])
    crafted[16:24] = struct.pack("<q", nnz)
    crafted[28:32] = struct.pack("<I", 1)
    crafted += struct.pack(f"<{n + 1}q", *([0] * n + [nnz])) + bytes(8 * n)
    variants.append(bytes(crafted))
    for _ in range(80):
        b = bytearray(good)
        for _ in range(rng.randint(1, 6)):
            b[rng.randrange(len(b))] = rng.randrange(256)
        variants.append(bytes(b))
    for i, b in enumerate(variants):
        p = tmp_path / f"v{i}.gcsr"
        p.write_bytes(b)
        paths.append(str(p))
    res = _run(driver, "csr", *paths)
    assert int(res[0][0]) == 0
    assert all(int(r[0]) in (0, -1, -3, -8) for r in res)


@pytest.mark.parametrize("n,d,seed", [(0, 4, 1), (1, 4, 1), (2, 1, 3), (1000, 8, 7), (5000, 16, 42)])
def test_generator(driver, n, d, seed):
    (st, nnz, _), = _run(driver, "gen", str(n), str(d), str(seed))
    assert int(st) == 0 and 0 <= int(nnz) <= n * d


def test_oracles_under_sanitizers(tmp_path):
    """The CPU oracles (oracle/gcolor_oracle.c every mode, oracle/gcolor_omp.c on 1-4 threads)
    under ASan+UBSan on 60 seeded random directed / symmetric multigraphs with self-loops and
    hubs, the OpenMP restatement cross-checked against the single-thread oracle (colours, rounds
    of colouring, every per-round record) inside the driver."""
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    exe = str(tmp_path / "orc_asan")
    cmd = ["gcc", "-std=c11", "-O1", "-g", "-fopenmp", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", os.path.join(REPO, "tests", "host_asan", "oracle_driver.c"),
           os.path.join(REPO, "oracle", "gcolor_oracle.c"), os.path.join(REPO, "oracle", "gcolor_omp.c"), "-o", exe, "-lm"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _run(exe, "60")
    assert out[-1] == ["ok", "60", "graphs"]
