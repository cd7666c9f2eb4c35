"""Write the committed golden fixtures from the CPU restatement (run in the build container).

    python tests/golden/make_golden.py

Fixtures are data only: the generating inputs are seeded synthetic frames
(my_orb_slam2_amd.synth), recorded by seed and SHA-256; outputs are either stored in full
(small frames, .npz) or as SHA-256 digests (full-size KITTI stereo pairs).
"""
import hashlib
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import oracle  # noqa: E402
from my_orb_slam2_amd import synth  # noqa: E402

OUT = ROOT / "tests" / "golden"
MBF, FX = 386.1448, 718.856


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    cases = {}
    # small frame, outputs in full
    img = synth.frame(42, 320, 240)
    e = oracle.OracleExtractor(500, 1.2, 8, 20, 7)
    k, d = e(img)
    np.savez_compressed(OUT / "small_320x240_seed42.npz", keypoints=k, descriptors=d)
    cases["small_320x240_seed42"] = {"input": ["frame", 42, 320, 240], "input_sha256": sha(img),
                                     "params": [500, 1.2, 8, 20, 7], "n": int(len(k))}
    # KITTI stereo pairs, digests
    mb = float(np.float32(MBF) / np.float32(FX))
    for seed in (0, 1):
        L, R = synth.stereo_pair(seed)
        ol = oracle.OracleExtractor(2000, 1.2, 8, 20, 7)
        orr = oracle.OracleExtractor(2000, 1.2, 8, 20, 7)
        kl, dl = ol(L)
        kr, dr = orr(R)
        u, dep, nv = oracle.stereo_match(ol, orr, len(kl), MBF, mb)
        cases[f"kitti_stereo_seed{seed}"] = {
            "input": ["stereo_pair", seed, 1241, 376], "input_sha256": [sha(L), sha(R)],
            "params": [2000, 1.2, 8, 20, 7], "mbf": MBF, "mb": mb,
            "n_left": int(len(kl)), "n_right": int(len(kr)), "n_valid": int(nv),
            "sha256": {"kps_left": sha(kl), "desc_left": sha(dl), "kps_right": sha(kr),
                       "desc_right": sha(dr), "uRight": sha(u), "depth": sha(dep)}}
    # edge images, digests
    for name, img in synth.edge_cases().items():
        e = oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
        k, d = e(img)
        cases[f"edge_{name}"] = {"input": ["edge", name], "input_sha256": sha(img),
                                 "params": [1000, 1.2, 8, 20, 7], "n": int(len(k)),
                                 "sha256": {"kps": sha(k),
                                            "desc": sha(d) if d is not None else None}}
    (OUT / "fixtures.json").write_text(json.dumps(cases, indent=1) + "\n")
    print(json.dumps({k: v.get("n", v.get("n_left")) for k, v in cases.items()}))


if __name__ == "__main__":
    main()
