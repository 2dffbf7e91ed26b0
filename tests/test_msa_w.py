"""CPU: `pafreport -w` — the multi-FASTA MSA of the last query run (pafreport.cpp:382-421, 447-450;
GapAssem.cpp GASeq::setGap :212-233, GSeqAlign(s1,s2) :605-641, addAlign :645-692, injectGap
:720-753, writeMSA :1039-1046) built by the product's closed form (pw_msa_layout.cpp: the query's
gap profile is the elementwise max over the alignments, target-only bases left-packed) against the
oracle's literal progressive merge (oracle/pafreport_oracle.c msa_*), byte for byte.

The layout is host work (no kernel touches it), so this runs through the host batch API
(pw_batch_write_msa); the CLI's `-w` plumbing, including its error exits, is compared on the GPU
in test_gpu_parity.py."""
import os

import pytest

import pwasm_amd as pw
from conftest import ORACLE, SYNTH, run, synth_paf
from test_gpu_parity import query_end_case

PW_E_ARG = -1  # include/pwasm_amd.h
FLAGS = {"-G": pw.FLAG_G, "-F": pw.FLAG_F, "-C": pw.FLAG_C, "-N": pw.FLAG_N}


def msa_same(fa, paf, tmp_path, flags=(), paths=("closed", "replay")):
    want = tmp_path / "oracle.mfa"
    rc, _, err = run([ORACLE, *flags, "-r", fa, "-w", want, "-o", tmp_path / "oracle.txt", paf])
    assert rc == 0, err
    bits = pw.FLAG_W
    for f in flags:
        bits |= FLAGS[f]
    a = want.read_bytes()
    batch = pw.HostBatch(fa, paf, bits)
    for mode in paths:  # the closed form must apply (no silent fallback), and the replay agrees
        got = tmp_path / f"hip_{mode}.mfa"
        os.environ["PW_MSA_PATH"] = mode
        try:
            assert batch.write_msa(str(got)) == 0, mode
        finally:
            os.environ.pop("PW_MSA_PATH", None)
        b = got.read_bytes()
        if a != b:
            x, y = a.decode().splitlines(), b.decode().splitlines()
            for i, (u, v) in enumerate(zip(x, y)):
                if u != v:
                    pytest.fail(f"{mode}: first difference at line {i}:\noracle: {u!r}\nhost:   {v!r}")
            pytest.fail(f"{mode}: length differs: oracle {len(x)} lines, host {len(y)} lines")
    return a


def big_run(tmp_path, seed, extra=()):
    """Two queries with hundreds of alignments each: the last run merges ~300 alignments."""
    fa, paf = str(tmp_path / "r.fa"), str(tmp_path / "r.paf")
    rc, _, err = run([SYNTH, "paf", "--config", 0, "--seed", seed, "--ncds", 2, "--recs", 300,
                      "--fa", fa, "--paf", paf, *extra])
    assert rc == 0, err
    return fa, paf


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6])
def test_edge_mix(built, tmp_path, seed):
    fa, paf = synth_paf(tmp_path, 0, seed=seed)
    out = msa_same(fa, paf, tmp_path)
    assert out.count(b">") >= 2


def test_no_msa_in_full_genome_mode(built, tmp_path):
    """-w with -F: the reference exits with "can only generate MSA for -G mode!"
    (pafreport.cpp:265-269), so the batch API builds no MSA there and pw_batch_write_msa refuses."""
    fa, paf = synth_paf(tmp_path, 2, seed=3, scale=0.01)
    rc, _, err = run([ORACLE, "-F", "-r", fa, "-w", tmp_path / "o.mfa", "-o", tmp_path / "o.txt", paf])
    assert rc == 1 and b"can only generate MSA for -G mode!" in err
    batch = pw.HostBatch(fa, paf, pw.FLAG_W | pw.FLAG_F)
    assert batch.write_msa(str(tmp_path / "b.mfa")) == PW_E_ARG


def test_cfg1(built, tmp_path):
    fa, paf = synth_paf(tmp_path, 1)
    msa_same(fa, paf, tmp_path)


@pytest.mark.parametrize("flags", [["-G", "-C"], ["-G"], ["-G", "-N"]])
def test_cfg2_modes(built, tmp_path, flags):
    fa, paf = synth_paf(tmp_path, 2, seed=3, scale=0.05)
    msa_same(fa, paf, tmp_path, flags)


@pytest.mark.parametrize("seed,extra", [(7, ()), (8, ("--rev", 1.0)), (9, ("--rev", 0.0)),
                                        (10, ("--longindel", 0.3, "--err", 0.05))])
def test_long_runs(built, tmp_path, seed, extra):
    fa, paf = big_run(tmp_path, seed, extra)
    out = msa_same(fa, paf, tmp_path)
    assert out.count(b">") > 100


def test_indels_at_query_ends(built, tmp_path):
    fa, paf = query_end_case(tmp_path)
    out = msa_same(fa, paf, tmp_path)
    assert out.count(b">") == 5  # the query row + 4 targets


def test_only_the_last_run_of_a_repeated_query(built, tmp_path):
    """qa, qb, qa: the refseq GASeq is rebuilt on every query switch (rseqs is never filled,
    pafreport.cpp:341-351), so the MSA holds the last qa run only."""
    fa, paf = query_end_case(tmp_path)
    lines = open(paf).read().splitlines(True)
    qb = "\t".join(map(str, ["qb", 24, 0, 24, "+", "tb", 100, 0, 24, 24, 24, 60, "NM:i:0", "AS:i:9", "cg:Z:24M", "cs:Z::24"])) + "\n"
    p = tmp_path / "switch.paf"
    p.write_text("".join(lines[:2]) + qb + "".join(lines[2:]))
    out = msa_same(fa, str(p), tmp_path)
    assert out.count(b">") == 3 and b">t3" in out and b">t1" not in out
