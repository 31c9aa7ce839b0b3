"""Randomised parity stress of the global form's span groups (kMediumSpans): bucket-overflow runs of
several sizes, loads and shapes, HIP against the oracle (GPU box; not part of the pytest suite)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.pyoracle import oracle_binding  # noqa: E402
from testground_amd import _abi as A  # noqa: E402
from tests import scenarios as S  # noqa: E402

hip, orc = A.hip_library(), oracle_binding()
cases = [(1500, 40), (2048, 120), (3000, 60), (4096, 30), (5000, 100), (8192, 50), (2600, 200), (6000, 70)]
for k, (n, per) in enumerate(cases):
    t = time.time()
    kc = []
    a = S.run_bucket_overflow(hip, 10 + k, n_inst=n, per_sender=per, counters=kc)
    b = S.run_bucket_overflow(orc, 10 + k, n_inst=n, per_sender=per)
    S.assert_same(a, b)
    print(f"n={n} per_sender={per}: HIP = oracle; long_emit {kc[-1]['long_emit']} long_tb {kc[-1]['long_tb']} "
          f"({time.time() - t:.1f} s)", flush=True)
print("span stress ok")
