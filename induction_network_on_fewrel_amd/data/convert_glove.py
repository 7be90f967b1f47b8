"""GloVe dimension-truncation CLI (reference ``util/convert_glove_vec.py:3-23``).

The reference script reads ``../data/glove.6B.50d.json`` and writes ``../data/glove.6B.5d.json``
(first 5 dims of every vector, words lower-cased) -- the file its ``train.py:25`` loads.  Same defaults
here, relative to the working directory, with the paths and width as options:

    python -m induction_network_on_fewrel_amd.data.convert_glove [--input F] [--output F] [--dim K]
"""
from __future__ import annotations

import argparse
import os
import sys

from .fewrel import truncate_word_vectors


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--input", default="./data/glove.6B.50d.json")
    ap.add_argument("--output", default="")
    ap.add_argument("--dim", type=int, default=5)
    a = ap.parse_args(argv)
    out = a.output or os.path.join(os.path.dirname(a.input) or ".", f"glove.6B.{a.dim}d.json")
    if not os.path.exists(a.input):
        print(f"convert_glove: {a.input} not found", file=sys.stderr)
        return 1
    truncate_word_vectors(a.input, out, a.dim)
    print(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
