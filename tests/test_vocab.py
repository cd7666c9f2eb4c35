"""DBoW2 vocabulary path (Frame::ComputeBoW): the restatement against an independent plain
Python reading (CPU), and the GPU descent + vectors against the restatement (gpu)."""
import numpy as np
import pytest

from my_orb_slam2_amd import synth


def hd(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def parse_vocab(path):
    lines = [l for l in open(path).read().split("\n") if l.strip()]
    k, L, sc, wt = (int(x) for x in lines[0].split())
    nodes = [dict(parent=0, leaf=0, desc=np.zeros(32, np.uint8), w=0.0, children=[], word=0)]
    nw = 0
    for ln in lines[1:]:
        t = ln.split()
        n = dict(parent=int(t[0]), leaf=int(t[1]), desc=np.array([int(x) for x in t[2:34]], np.uint8),
                 w=float(t[34]), children=[], word=0)
        if n["leaf"] > 0:
            n["word"] = nw
            nw += 1
        nodes[n["parent"]]["children"].append(len(nodes))
        nodes.append(n)
    return k, L, sc, wt, nodes


def transform_py(path, desc, levelsup):
    k, L, sc, wt, nodes = parse_vocab(path)
    bow, fv, words, nids = {}, {}, [], []
    for i, f in enumerate(desc):
        nid_level = L - levelsup
        nid = 0 if nid_level <= 0 else None
        cur, level = 0, 0
        while True:
            level += 1
            ch = nodes[cur]["children"]
            best, bd = ch[0], hd(f, nodes[ch[0]]["desc"])
            for c in ch[1:]:
                d = hd(f, nodes[c]["desc"])
                if d < bd:
                    best, bd = c, d
            cur = best
            if level == nid_level:
                nid = cur
            if not nodes[cur]["children"]:
                break
        nid = cur if nid is None else nid
        words.append(nodes[cur]["word"])
        nids.append(nid)
        w = nodes[cur]["w"]
        if w > 0:
            if wt in (0, 1):
                bow[nodes[cur]["word"]] = bow.get(nodes[cur]["word"], 0.0) + w
            else:
                bow.setdefault(nodes[cur]["word"], w)
            fv.setdefault(nid, []).append(i)
    must = sc != 5
    if wt in (0, 1) and bow and not must:
        nd = float(len(bow))
        bow = {a: b / nd for a, b in bow.items()}
    if must:
        keys = sorted(bow)
        if sc != 1:
            norm = 0.0
            for a in keys:
                norm += abs(bow[a])
        else:
            norm = 0.0
            for a in keys:
                norm += bow[a] * bow[a]
            norm = np.sqrt(norm)
        if norm > 0:
            bow = {a: b / norm for a, b in bow.items()}
    return words, nids, bow, fv


@pytest.mark.parametrize("k,L,sc,wt,levelsup", [(4, 3, 0, 0, 1), (3, 3, 1, 1, 2), (5, 2, 5, 0, 1),
                                                (3, 3, 0, 2, 4), (4, 2, 5, 3, 0)])
def test_vocab_oracle_crosscheck(tmp_path, k, L, sc, wt, levelsup):
    from oracle.matcher import OracleVocabulary
    path = tmp_path / "voc.txt"
    synth.write_vocabulary(path, k=k, L=L, seed=k * 10 + L, scoring=sc, weighting=wt,
                           stop_frac=0.2)
    desc = np.random.default_rng(k).integers(0, 256, (120, 32), dtype=np.uint8)
    v = OracleVocabulary(path)
    w, n, (bw, bv), (fn, fo, ff) = v.transform(desc, levelsup)
    pw, pn, pbow, pfv = transform_py(path, desc, levelsup)
    np.testing.assert_array_equal(w, pw)
    np.testing.assert_array_equal(n, pn)
    np.testing.assert_array_equal(bw, sorted(pbow))
    np.testing.assert_array_equal(bv.view(np.int64), np.array([pbow[a] for a in sorted(pbow)]).view(np.int64))
    np.testing.assert_array_equal(fn, sorted(pfv))
    np.testing.assert_array_equal(ff, np.concatenate([pfv[a] for a in sorted(pfv)]) if pfv else [])


def test_vocab_first_min_tie(tmp_path):
    """Two children with the same descriptor: the first one always wins (d < best_d)."""
    from oracle.matcher import OracleVocabulary
    z = " ".join(["0"] * 32)
    o = " ".join(["255"] * 32)
    (tmp_path / "v.txt").write_text(f"2 1 0 0\n0 1 {z} 1.5\n0 1 {z} 2.5\n0 1 {o} 3.0\n")
    v = OracleVocabulary(tmp_path / "v.txt")
    w, n, (bw, bv), _ = v.transform(np.zeros((3, 32), np.uint8), 0)
    assert list(w) == [0, 0, 0] and list(bw) == [0] and bv[0] == 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("k,L,sc,wt,levelsup", [(10, 3, 0, 0, 2), (10, 4, 1, 1, 2),
                                                (6, 4, 5, 2, 3), (8, 3, 0, 3, 1)])
def test_vocab_gpu(tmp_path, oracle_mod, orbx_lib, gpu, k, L, sc, wt, levelsup):
    from oracle.matcher import OracleVocabulary, bow_score_l1 as o_score
    from my_orb_slam2_amd import Vocabulary, bow_score_l1
    path = tmp_path / "voc.txt"
    synth.write_vocabulary(path, k=k, L=L, seed=k + L, scoring=sc, weighting=wt)
    rng = np.random.default_rng(L)
    descs = [rng.integers(0, 256, (n, 32), dtype=np.uint8) for n in (2000, 1000, 1, 0)]
    gv, ov = Vocabulary.load_text(path), OracleVocabulary(path)
    bows = []
    for d in descs:
        w, n, (bw, bv), fv = gv.transform(d, levelsup)
        ow, on, (obw, obv), (ofn, ofo, off) = ov.transform(d, levelsup)
        np.testing.assert_array_equal(w, ow)
        np.testing.assert_array_equal(n, on)
        np.testing.assert_array_equal(bw, obw)
        np.testing.assert_array_equal(bv.view(np.int64), obv.view(np.int64))
        np.testing.assert_array_equal(fv.node_id, ofn)
        np.testing.assert_array_equal(fv.off, ofo)
        np.testing.assert_array_equal(fv.feat, off)
        bows.append((bw, bv))
    assert bow_score_l1(bows[0], bows[1]) == o_score(bows[0], bows[1])


@pytest.mark.gpu
def test_bow_db_score_gpu(tmp_path, oracle_mod, orbx_lib, gpu):
    """KeyFrameDatabase scoring pass: shared-word counts and (float) L1 scores of 300
    keyframe BowVectors against one query, vs the restated L1Scoring::score."""
    from oracle.matcher import OracleVocabulary, bow_score_l1 as o_score
    from my_orb_slam2_amd.vocabulary import bow_db_score
    path = tmp_path / "voc.txt"
    synth.write_vocabulary(path, k=10, L=3, seed=5)
    ov = OracleVocabulary(path)
    rng = np.random.default_rng(0)
    base = rng.integers(0, 256, (800, 32), dtype=np.uint8)
    q = ov.transform(base, 2)[2]
    kfs = []
    for i in range(300):
        d = base.copy() if i % 3 == 0 else rng.integers(0, 256, (rng.integers(0, 900), 32), dtype=np.uint8)
        if i % 3 == 0:
            d[rng.random(len(d)) < 0.5] = rng.integers(0, 256, 32, dtype=np.uint8)
        kfs.append(ov.transform(d, 2)[2])
    common, score = bow_db_score(q, kfs)
    for i, b in enumerate(kfs):
        assert common[i] == len(np.intersect1d(q[0], b[0]))
        assert score[i] == np.float32(o_score(q, b)), i
