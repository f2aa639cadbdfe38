"""Generate tests/golden/golden.json from the CPU oracles (run in this container).

What is pinned where (see DESIGN.md "Oracle and parity"):
  * blake3_kat.json — published BLAKE3 vectors (hand-entered, not generated):
    pins the BLAKE3 restatement.
  * host_kat.json — published SHA-256 / HMAC / HKDF / AES-256 / GCM /
    CRC-32C / secp256k1 vectors (hand-entered): pins host_oracle.py.
  * golden.json (this script) — zfec encoding matrices and the level-4/8/12
    encodings of the reference's own sample files (tests/samples of the
    reference, copied under samples/): sizes, EncodeInfo, bao hash and the
    BLAKE3 digest of the whole encoded stream.  Produced by the C oracle and
    cross-checked here against the independent Python oracle (pyoracle.py).
    The zfec-rs crate is absent from the container, so the parity bytes are
    "parity unpinned" against the real crate; these vectors pin our two
    oracles and the GPU path to each other and to the fec.c construction.
Usage: python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from oracle import oracle as O  # noqa: E402
from oracle import host_oracle as H  # noqa: E402
from oracle import pyoracle as P  # noqa: E402

HERE = Path(__file__).resolve().parent
SAMPLES = ["contract.rgbc", "content.png", "code.tar"]
# Fixed ECIES material for the host-stage levels: the receiver's secret key and
# the two values ecies::encrypt would draw from thread_rng (injected).
GOLDEN_SK = H.sha256(b"carbonado-amd golden receiver key")
GOLDEN_EPH = H.sha256(b"carbonado-amd golden ephemeral key")
GOLDEN_NONCE = H.sha256(b"carbonado-amd golden nonce")[:16]
HOST_LEVELS = (1, 2, 3, 14, 15)


def main() -> None:
    out: dict = {"generator": "tests/golden/make_golden.py (C oracle, cross-checked by pyoracle)"}
    mats = {}
    for k, m in [(4, 8), (8, 16), (3, 10), (2, 5)]:
        E = O.enc_matrix(k, m).tolist()
        assert E == P.enc_matrix(k, m)
        mats[f"{k}of{m}"] = [bytes(r).hex() for r in E]
    out["enc_matrix"] = mats
    samples = {}
    for name in SAMPLES:
        data = (HERE / "samples" / name).read_bytes()
        entry = {"input_len": len(data), "input_blake3": O.blake3(data).hex()}
        assert P.blake3(data) == O.blake3(data)
        for level in (4, 8, 12):
            enc, h, info = O.encode(data, level)
            if level in (8, 12):
                z, pad, C = P.zfec_encode(data)
                assert (pad, C) == (info["padding_len"], info["chunk_len"])
                if level == 8:
                    assert z == enc
                else:
                    pe, ph = P.bao_encode(z)
                    assert pe == enc and ph == h
            else:
                pe, ph = P.bao_encode(data)
                assert pe == enc and ph == h
            entry[f"level{level}"] = {
                "hash": h.hex(),
                "output_len": len(enc),
                "output_blake3": O.blake3(enc).hex(),
                "info": {k: (round(v, 6) if isinstance(v, float) else v) for k, v in info.items()},
            }
        pub = H.public_key(GOLDEN_SK)
        for level in HOST_LEVELS:
            enc, h, info = O.encode_full(data, level, pub, GOLDEN_EPH, GOLDEN_NONCE)
            assert O.decode_full(GOLDEN_SK, h, enc, info["padding_len"], level) == data
            entry[f"level{level}"] = {
                "hash": h.hex(),
                "output_len": len(enc),
                "output_blake3": O.blake3(enc).hex(),
                "info": {k: (round(v, 6) if isinstance(v, float) else v) for k, v in info.items()},
            }
        samples[name] = entry
    out["samples"] = samples
    out["ecies_material"] = {"secret_key": GOLDEN_SK.hex(), "ephemeral_sk": GOLDEN_EPH.hex(),
                             "nonce": GOLDEN_NONCE.hex(), "public_key": H.public_key(GOLDEN_SK).hex()}
    # small deterministic zfec/bao vectors (inputs from the shared generator)
    vec = []
    for n, seed in [(1, 1), (1000, 2), (4096, 3), (5000, 4), (12289, 5)]:
        d = O.fill_object(seed, 0, n).tobytes()
        z, pad, C = O.zfec_encode(d)
        b, h = O.bao_encode(z)
        vec.append({"n": n, "seed": seed, "padding": pad, "chunk_len": C,
                    "zfec_blake3": O.blake3(z).hex(), "bao_hash": h.hex(), "bao_len": len(b)})
    out["generated_vectors"] = vec
    (HERE / "golden.json").write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print("wrote", HERE / "golden.json")


if __name__ == "__main__":
    main()
