"""Tokenise local text into nanoGPT's uint16 ``train.bin`` / ``val.bin`` memmaps (reference
python/examples/nanogptddp/prepare_owt_dataset.py downloads OpenWebText and uses tiktoken; neither the network nor
tiktoken is assumed here).

    python prepare_data.py --input corpus.txt --out-dir data/   [--tokenizer path/to/tokenizer.json]

With ``--tokenizer`` a HuggingFace ``tokenizers`` JSON file is used (e.g. GPT-2's), otherwise a byte-level
tokenizer (vocab 256). Without ``--input`` a synthetic corpus is generated.
"""
import argparse
import os

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--input", default=None)
    ap.add_argument("--out-dir", default="data")
    ap.add_argument("--tokenizer", default=None)
    ap.add_argument("--val-fraction", type=float, default=0.0005)
    ap.add_argument("--synthetic-bytes", type=int, default=8 << 20)
    a = ap.parse_args()
    if a.input:
        with open(a.input, "rb") as f:
            raw = f.read()
    else:
        rng = np.random.default_rng(0)
        words = [bytes(rng.integers(97, 123, size=rng.integers(2, 9)).astype(np.uint8)) for _ in range(5000)]
        raw = b" ".join(words[i] for i in rng.integers(0, len(words), size=a.synthetic_bytes // 6))
    if a.tokenizer:
        from tokenizers import Tokenizer
        tok = Tokenizer.from_file(a.tokenizer)
        ids = np.array(tok.encode(raw.decode("utf-8", errors="replace")).ids, dtype=np.uint16)
    else:
        ids = np.frombuffer(raw, dtype=np.uint8).astype(np.uint16)
    n_val = max(1, int(len(ids) * a.val_fraction))
    os.makedirs(a.out_dir, exist_ok=True)
    ids[:-n_val].tofile(os.path.join(a.out_dir, "train.bin"))
    ids[-n_val:].tofile(os.path.join(a.out_dir, "val.bin"))
    print(f"train {len(ids) - n_val} tokens, val {n_val} tokens -> {a.out_dir}")


if __name__ == "__main__":
    main()
