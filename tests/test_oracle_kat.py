"""CPU: the oracle (oracle/pafreport_oracle.c) against the hand-derived known-answer tests
in tests/golden/kat (see tests/golden/make_kats.py for each derivation), plus the GapAssem
oracle against hand-derived layouts."""
import json
import os
import shutil
import struct

import pytest

from conftest import GA_ORACLE, KAT_DIR, ORACLE, run

CASES = sorted(d for d in os.listdir(KAT_DIR) if os.path.isdir(KAT_DIR / d))


def run_case(binary, case, tmp_path):
    src = KAT_DIR / case
    dst = tmp_path / case
    shutil.copytree(src, dst)
    spec = json.load(open(dst / "args.json"))
    rc, out, err = run([binary, *spec["args"]], cwd=dst)
    exp_out = open(src / "stdout", "rb").read()
    exp_err = open(src / "stderr", "rb").read()
    assert rc == spec["rc"], (rc, err)
    assert out == exp_out
    assert err == exp_err
    if "outfile" in spec:
        assert open(dst / spec["outfile"]).read() == spec["outfile_expected"]
    for name in spec.get("absent", []):  # option values the reference never opens (-s, -p, -m, -d)
        assert not (dst / name).exists(), name


@pytest.mark.parametrize("case", CASES)
def test_oracle_kat(built, case, tmp_path):
    run_case(ORACLE, case, tmp_path)


def write_pwl(path, rows):
    with open(path, "wb") as f:
        f.write(b"PWL1" + struct.pack("<I", len(rows)))
        for off, seq, ofs, clp5, clp3, rev in rows:
            f.write(struct.pack("<5i", off, len(seq), clp5, clp3, rev))
            f.write(seq.encode())
            f.write(struct.pack(f"<{len(ofs)}h", *ofs))


def read_pwc(path):
    b = open(path, "rb").read()
    assert b[:4] == b"PWC1"
    length, minoff, mincol, maxcol, clen, removed = struct.unpack_from("<6i", b, 4)
    p = 28
    cons = b[p:p + clen].decode()
    p += clen
    counts = struct.unpack_from(f"<{6 * length}i", b, p)
    p += 24 * length
    (nrows,) = struct.unpack_from("<I", b, p)
    return dict(length=length, minoff=minoff, mincol=mincol, maxcol=maxcol, cons=cons, removed=removed,
                counts=[counts[6 * i:6 * i + 6] for i in range(length)], nrows=nrows, raw=b)


# Hand-derived (GapAssem.cpp:551-591 toMSA, GapAssem.h:295-337 add*, :1048-1069 bestChar):
#   row0 offset 0 "ACGT" ofs [0,0,1,0]  -> cols A0 C1 -2 G3 T4
#   row1 offset 1 "CNGA" ofs [0,0,1,0]  -> cols C1 N2 -3 G4 A5
#   row2 offset 2 "-G"   ofs [0,0]      -> '-'2 (gap char counted as gap) G3
# col0 A:1 -> A; col1 C:2 -> C; col2 -:2 (row0 gap, row2 '-') N:1 -> '-' -> '*';
# col3 G:2 -:1 -> G; col4 T:1 G:1 -> tie, stable order A,C,G,T -> G; col5 A:1 -> A.
# consensus "AC*GGA", mincol 0, maxcol 5.
def test_gapassem_oracle_hand_layout(built, tmp_path):
    lay = tmp_path / "l.pwl"
    write_pwl(lay, [(0, "ACGT", [0, 0, 1, 0], 0, 0, 0), (1, "CNGA", [0, 0, 1, 0], 0, 0, 0),
                    (2, "-G", [0, 0], 0, 0, 0)])
    rc, _, err = run([GA_ORACLE, lay, tmp_path / "o.pwc"])
    assert rc == 0, err
    r = read_pwc(tmp_path / "o.pwc")
    assert r["cons"] == "AC*GGA"
    assert (r["mincol"], r["maxcol"], r["length"]) == (0, 5, 6)
    assert r["counts"][2] == (0, 0, 0, 0, 1, 2)
    assert r["counts"][4] == (0, 0, 1, 1, 0, 0)


# N and '-' tied at the max -> '-' (the qsort/tie loop of bestChar, GapAssem.cpp:1057-1066);
# N alone at the max -> 'N'; zero-coverage column inside [mincol,maxcol] -> exit 5.
def test_gapassem_oracle_ties_and_zero(built, tmp_path):
    lay = tmp_path / "t.pwl"
    write_pwl(lay, [(0, "NNA", [0, 0, 0], 0, 0, 0), (0, "-NA", [0, 0, 0], 0, 0, 0)])
    rc, _, err = run([GA_ORACLE, lay, tmp_path / "t.pwc"])
    assert rc == 0, err
    assert read_pwc(tmp_path / "t.pwc")["cons"] == "*NA"
    lay2 = tmp_path / "z.pwl"  # row1 starts one column after row0 ends -> empty column 3
    write_pwl(lay2, [(0, "ACG", [0, 0, 0], 0, 0, 0), (4, "TT", [0, 0], 0, 0, 0)])
    rc, _, err = run([GA_ORACLE, lay2, tmp_path / "z.pwc"])
    assert rc == 5
    assert err.startswith(b"WARNING: 0 coverage column 3 (mincol=0) found within alignment of 2 seqs!\n")
