"""ORACLE — test infrastructure only.

CPU restatements of the reference (JunyiPeng00/wespeaker_hubert) extraction +
scoring path.  Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg may import anything from here, and only as the *checker* or
as the timed CPU baseline — never as the product path.  The product
(`wespeaker_hubert_amd`) never imports this package and fails loudly when its
HIP library is missing.

Pinning status:
  * models_ref (ECAPA-TDNN, ResNet, ASTP/TSTP): pinned by golden fixtures made
    from the reference's own modules (tests/golden/make_golden.py).
  * scoring_ref (get_mean_std, EER, minDCF): pinned by golden fixtures made
    from the reference's own functions.
  * fbank_ref: restates torchaudio.compliance.kaldi.fbank (third-party,
    absent here) — **parity unpinned** against reference outputs; it is
    cross-checked against an independent float64 DFT formulation and against
    the reference's own C++ restatement read as text
    (runtime/core/frontend/fbank.h:138-198), which cannot be compiled here
    without a glog stand-in.
"""
