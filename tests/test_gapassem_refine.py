"""CPU: the closed form the GPU's refineMSA kernels implement (pw_msa.hip K6-K9)
against the GapAssem oracle's literal replay of GSeqAlign::refineMSA with removeConsGaps
(GapAssem.cpp:1143-1181: removeColumn :755-779 -> GASeq::removeBase :122-131, removeClipGaps
:522-549) on random layouts, clipped rows included.  The model below is test code only; the
product computes the same closed form on the GPU (test_gpu_parity.py::test_gapassem_remove_gaps*).

Closed form, with G(c) = consensus-gap columns in [mincol, c], O = offset - minoffset and
col(i) the layout column of base i (toMSA, GapAssem.cpp:568-588):
  offset' = offset - G(O);  ofs'[0] -= G(col(0)) - G(O);  ofs'[i] -= G(col(i)) - G(col(i-1))
then removeClipGaps moves ofs'[i <= clipL] into the offset and zeroes ofs'[i >= len - clipR]."""
import random
import struct

import pytest

from conftest import GA_ORACLE, run
from test_oracle_kat import read_pwc, write_pwl


def read_rows(pwc_raw, lens):
    p = 4 + 24
    length, _, _, _, clen, _ = struct.unpack_from("<6i", pwc_raw, 4)
    p += clen + 24 * length
    (n,) = struct.unpack_from("<I", pwc_raw, p)
    p += 4
    out = []
    for r in range(n):
        off, ng, _c5, _c3 = struct.unpack_from("<4i", pwc_raw, p)
        p += 16
        ofs = list(struct.unpack_from(f"<{lens[r]}h", pwc_raw, p))
        p += 2 * lens[r]
        out.append((off, ng, ofs))
    return out


def read_clips(pwc_raw, lens):
    """(clp5, clp3) of every row of a PWC1 result."""
    p = 4 + 24
    length, _, _, _, clen, _ = struct.unpack_from("<6i", pwc_raw, 4)
    p += clen + 24 * length + 4
    out = []
    for n in lens:
        out.append(struct.unpack_from("<2i", pwc_raw, p + 8))
        p += 16 + 2 * n
    return out


def model(rows, res, clip_gaps=True):
    """Closed-form refineMSA row edits from the oracle's consensus columns (clip_gaps=False: stop
    before removeClipGaps, as pw_msa_refine with keep_clip_gaps)."""
    minoff = res["minoff"]
    lo, hi = res["mincol"], res["maxcol"]
    cons_gap = set()
    if lo >= 0:
        for c in range(lo, hi + 1):
            cnt = res["counts"][c]
            m = max(cnt)
            bi = cnt.index(m)
            ch = "ACGTN-"[bi]
            if bi == 4 and cnt[5] == m:
                ch = "-"
            if ch == "-":
                cons_gap.add(c)
    G = []
    acc = 0
    for c in range(res["length"]):
        acc += c in cons_gap
        G.append(acc)

    def g(c):
        return 0 if c < 0 else G[min(c, len(G) - 1)]

    out = []
    for off, seq, ofs, clp5, clp3, rev in rows:
        O = off - minoff
        numgaps = sum(ofs)
        new_off = off - g(O)
        new = []
        col = O - 1
        for i, x in enumerate(ofs):
            prev = O if i == 0 else col
            col += 1 + max(x, 0)
            dec = g(col) - g(prev)
            new.append(x - dec)
            numgaps -= dec
        cl, cr = (clp3, clp5) if rev else (clp5, clp3)
        if not clip_gaps:
            out.append((new_off, numgaps, new))
            continue
        dl = dr = 0
        for i in range(len(new)):
            if i <= cl:
                dl += new[i]
                new[i] = 0
            elif i >= len(new) - cr:
                dr += new[i]
                new[i] = 0
        out.append((new_off + dl, numgaps - dl - dr, new))
    return out


def random_layout(rng, nrows, clip, dels=False):
    """Random rows (offset, seq, ofs, clp5, clp3, rev); dels: some deleted bases (ofs -1)."""
    rows = []
    for r in range(nrows):
        n = rng.randint(5, 40)
        seq = "".join(rng.choice("ACGTACGTN-") for _ in range(n))
        ofs = [rng.choice([0, 0, 0, 0, 1, 2, 3] + ([-1] if dels else [])) for _ in range(n)]
        c5 = rng.randint(0, 6) if clip else 0
        c3 = rng.randint(0, 6) if clip else 0
        rows.append((rng.randint(0, 25), seq, ofs, c5, c3, r % 2))
    return rows


@pytest.mark.parametrize("seed", range(40))
def test_closed_form_matches_oracle(built, tmp_path, seed):
    rng = random.Random(100 + seed)
    rows = random_layout(rng, rng.randint(2, 14), clip=seed % 2 == 1)
    lay = tmp_path / "l.pwl"
    write_pwl(lay, rows)
    rc, _, err = run([GA_ORACLE, lay, tmp_path / "o.pwc", "--remove-gaps", "--no-refine-clipping"])
    if rc != 0:  # zero-coverage / trimmed rows: nothing to compare
        assert rc in (1, 5), err
        return
    res = read_pwc(tmp_path / "o.pwc")
    got = read_rows(res["raw"], [len(r[1]) for r in rows])
    assert got == model(rows, res)
    # the consensus drops exactly the gap columns
    rc2, _, _ = run([GA_ORACLE, lay, tmp_path / "k.pwc", "--no-refine-clipping"])
    keep = read_pwc(tmp_path / "k.pwc")["cons"]
    assert res["cons"] == keep.replace("*", "")
    assert res["removed"] == keep.count("*")
