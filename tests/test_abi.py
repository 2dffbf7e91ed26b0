"""CPU: the C-ABI library loads and exports every function include/pwasm_amd.h declares; the
host pre-pass (pw_pack_cs) packs cs strings the way pafreport.cpp:536-626 reads them; CLI
argument errors (which return before any device work) match the reference's messages."""
import re
import subprocess

import pytest

import pwasm_amd as pw
from conftest import CLI, REPO
from test_oracle_kat import run_case

HEADER = REPO / "include" / "pwasm_amd.h"


def declared_functions():
    txt = HEADER.read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w \*]*?\b(pw_\w+)\s*\(", txt, flags=re.M)))


def test_library_loads_and_exports_every_declared_symbol(built):
    L = pw.lib()
    names = declared_functions()
    assert "pw_report_events" in names and "pw_msa_columns" in names and "pw_pack_cs" in names
    nm = subprocess.run(["nm", "-D", "--defined-only", str(pw.LIB_PATH)], stdout=subprocess.PIPE, text=True).stdout
    exported = set(re.findall(r" T (pw_\w+)", nm))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    for n in names:
        assert n in pw._SIGS, f"{n} has no ctypes signature"
        getattr(L, n)
    assert "gfx950" in pw.version()


def test_pack_cs_basic(built):
    rc, ops, lits, tot, _ = pw.pack_cs(":4*ga:10-t:15", 0, 30)
    assert rc == pw.PW_CS_OK
    M = lambda t, n: (t << 30) | n
    assert ops == [M(0, 4), M(1, 1), M(0, 10), M(2, 1), M(0, 15)]
    assert lits == b"GAT"
    assert (tot.q_total, tot.t_total, tot.n_events_max) == (30, 31, 2)


def test_pack_cs_drops_zero_matches_and_uppercases(built):
    rc, ops, lits, tot, _ = pw.pack_cs(":0*ga:0*tc+acg:2-ttt", 5, 30)
    assert rc == 0
    assert [o >> 30 for o in ops] == [1, 1, 3, 0, 2]
    assert lits == b"GATCTTT"
    assert (tot.q_total, tot.t_total) == (7, 7)


@pytest.mark.parametrize("cs,qlen,code,pos", [
    (":4~gt10ag:26", 30, pw.PW_CS_SPLICED, 3),
    (":x", 30, pw.PW_CS_PARSE, 1),
    (":4=a", 30, pw.PW_CS_UNHANDLED, 3),
    (":4-:5", 30, pw.PW_CS_EMPTY, 3),
    (":4+", 30, pw.PW_CS_EMPTY, 3),
    (":31", 30, pw.PW_CS_BOUNDS, 3),
    (":29+aa", 30, pw.PW_CS_BOUNDS, 6),
    (":4*g", 30, pw.PW_CS_PARSE, 3),
])
def test_pack_cs_errors(built, cs, qlen, code, pos):
    rc, _, _, _, epos = pw.pack_cs(cs, 0, qlen)
    assert rc == code
    assert epos == pos


def test_pack_cs_sub_at_query_end_is_left_to_the_device(built):
    # '*' at q_pos == L reads the query's NUL terminator in the reference -> base-mismatch
    # error produced by the GPU check, not a host bounds error
    rc, ops, _, _, _ = pw.pack_cs(":30*ga", 0, 30)
    assert rc == pw.PW_CS_OK and len(ops) == 2


@pytest.mark.parametrize("case", ["cli_no_r", "cli_G_F", "cli_C_N", "cli_bad_opt"])
def test_cli_argument_errors(built, case, tmp_path):
    run_case(CLI, case, tmp_path)


@pytest.mark.parametrize("max_qlen,n_queries,want", [
    (5000, 1000, 13),        # cfg2: 13 position bits + 10 query bits
    (3000, 200, 12),         # cfg3 gene panel
    (5_000_000, 100, 23),    # cfg4 Mb contigs
    (4096, 1, 13),           # a position may equal the query length (a deletion at the end)
    (0, 0, 1),
    (1000, 1 << 25, 0),      # 10 + 25 bits: 32-byte records
    (1 << 31, 2, 0),
])
def test_hot_pbits_rule(built, max_qlen, n_queries, want):
    """pw_report_hot_pbits: when the 16-byte event record (query index and position in one word)
    applies, and how many position bits it takes."""
    import pwasm_amd as pw
    assert pw.lib().pw_report_hot_pbits(max_qlen, n_queries) == want
