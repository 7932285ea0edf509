"""Copy the reference's S&P 500 daily closes into a committed fixture.

tools/market_data/stooq_snp.npy (9167 x 1 float64, the C4 workload's price
table) is DATA the reference already holds; the GPU box has no
/root/reference, so the C4 bench and the full-size market tests read it from
tests/golden/stooq_snp.npz.  Loaded with allow_pickle=False (plain array file).

    python tests/golden/make_market_data.py
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/tools/market_data"


def main():
    snp = np.load(os.path.join(SRC, "stooq_snp.npy"), allow_pickle=False)
    assert snp.shape == (9167, 1) and snp.dtype == np.float64
    np.savez_compressed(os.path.join(HERE, "stooq_snp.npz"), prices=snp)
    print("wrote stooq_snp.npz", snp.shape)


if __name__ == "__main__":
    main()
