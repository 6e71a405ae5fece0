"""Adds published BER curves to published_ber.json (numbers copied as data
from the reference's CSVs; build container only, needs /root/reference).

threshold_init:
soft_hardinit_plot (sparc_ldpc.py:1435-1590) with L=M=512 P=4 r_sparc=1 T=64,
802.16 rate 5/6 over all 512 sections, soft_iter=2, sigma = linspace(0.9, 1.4, 10):
  thresholdinit_LM512Rsparc1P4_stndrd80216_Rldpc5_6_it2_rep200_threshold0_6.csv (two runs)
  shinit_LM512Rsparc1P4_stndrd80216_Rldpc5_6_it2_rep100_threshold0_6.csv
  shinit_LM512Rsparc1P4_stndrd80216_Rldpc5_6_it2_rep100_threshold0_8.csv
"""
import json
import os

REF = "/root/reference/ldpc"
HERE = os.path.dirname(os.path.abspath(__file__))
FILES = {
    "thresholdinit_LM512Rsparc1P4_stndrd80216_Rldpc5_6_it2_rep200_threshold0_6.csv": 0.6,
    "shinit_LM512Rsparc1P4_stndrd80216_Rldpc5_6_it2_rep100_threshold0_6.csv": 0.6,
    "shinit_LM512Rsparc1P4_stndrd80216_Rldpc5_6_it2_rep100_threshold0_8.csv": 0.8,
}


def vec(s):
    return [float(x) for x in s.strip().strip("[]").split()]


def parse(path):
    runs, cur = [], None
    for line in open(path):
        line = line.strip()
        if not line:
            continue
        if line.startswith("EbN0_dB"):
            cur = dict(EbN0_dB=[], BER_amp=[], BER_ldpc=[], BER_plain=[])
            runs.append(cur)
            continue
        # EbN0_dB,"[a b]","[c d]",plain  (numpy array reprs, no quotes in these files)
        head, rest = line.split(",", 1)
        a_end = rest.index("]")
        amp = rest[:a_end + 1]
        rest = rest[a_end + 2:]
        l_end = rest.index("]")
        ldpc = rest[:l_end + 1]
        plain = rest[l_end + 2:]
        cur["EbN0_dB"].append(float(head))
        cur["BER_amp"].append(vec(amp))
        cur["BER_ldpc"].append(vec(ldpc))
        cur["BER_plain"].append(float(plain))
    return runs


def parse_soft_hard(path):
    """EbN0VsBER_soft_hard_100_4.csv: a soft block (EbN0_dB, BER_sparc,
    BER_ldpc_soft [2], BER_amp_soft [3]) then a hard block (EbN0_dB, BER_sparc,
    BER_ldpc_hard, BER_amp_hard [2])."""
    out, cur = {}, None
    for line in open(path):
        line = line.strip()
        if not line:
            continue
        if line.startswith("EbN0_dB"):
            cur = "soft" if "soft" in line else "hard"
            out[cur] = dict(EbN0_dB=[], BER_sparc=[], BER_ldpc=[], BER_amp=[])
            continue
        head, sp_, rest = line.split(",", 2)
        d = out[cur]
        d["EbN0_dB"].append(float(head))
        d["BER_sparc"].append(float(sp_))
        if cur == "soft":
            e = rest.index("]")
            d["BER_ldpc"].append(vec(rest[:e + 1]))
            d["BER_amp"].append(vec(rest[e + 2:]))
        else:
            ldpc, amp = rest.split(",", 1)
            d["BER_ldpc"].append(float(ldpc))
            d["BER_amp"].append(vec(amp))
    return out


def main():
    p = os.path.join(HERE, "published_ber.json")
    pub = json.load(open(p))
    # soft_hard_plot (sparc_ldpc.py:1285-1432, __main__ :1672-1674): L=768 M=512
    # P=1.8 r_sparc=1 T=64, 802.16 5/6 with sec=569 (z=213), soft_iter=2,
    # sigma = linspace(0.8, 0.4, 10), MIN_ERRORS = MAX_BLOCKS = 100
    pub["soft_hard"] = dict(
        config=dict(L=768, M=512, P=1.8, r_sparc=1, T=64, standard="802.16", r_ldpc="5/6", sec=569, soft_iter=2,
                    sigma=[0.8, 0.4, 10], MIN_ERRORS=100, MAX_BLOCKS=100,
                    file="EbN0VsBER_soft_hard_100_4.csv"),
        **parse_soft_hard(os.path.join(REF, "EbN0VsBER_soft_hard_100_4.csv")))
    runs = []
    for f, thr in FILES.items():
        for r in parse(os.path.join(REF, f)):
            r["file"] = f
            r["threshold"] = thr
            runs.append(r)
    pub["threshold_init"] = dict(
        config=dict(L=512, M=512, P=4, r_sparc=1, T=64, standard="802.16", r_ldpc="5/6", sections=512,
                    soft_iter=2, sigma=[0.9, 1.4, 10], source="sparc_ldpc.py:1435-1590 soft_hardinit_plot"),
        runs=runs)
    with open(p, "w") as fh:
        json.dump(pub, fh, indent=1)
    print(f"{len(runs)} runs")


if __name__ == "__main__":
    main()
