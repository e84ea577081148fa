"""Counts host<->device copies of one describe() step by calling line
(Tensor.cpu / .item / .tolist / .to(device) / torch.tensor(device=)).
    python tools/sync_census.py [rows]"""
import collections
import sys
import traceback

sys.path.insert(0, 'spark-df-profiling_amd')
sys.path.insert(0, '.')
import torch  # noqa: E402

import bench  # noqa: E402
from spark_df_profiling import describe  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10 ** 8
t = bench.make_c3_shard(rows, 0, 1, torch.device('cuda'))
describe(t, plots=False)
torch.cuda.synchronize()
census = collections.Counter()


def site():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if 'spark_df_profiling' in fr.filename:
            return '%s:%d %s' % (fr.filename.split('/')[-1], fr.lineno, fr.name)
    return '?'


def wrap(owner, name, pred=lambda *a, **k: True):
    orig = getattr(owner, name)

    def f(*a, **k):
        if pred(*a, **k):
            census[(name, site())] += 1
        return orig(*a, **k)
    setattr(owner, name, f)


wrap(torch.Tensor, 'cpu', lambda self, *a, **k: self.is_cuda)
wrap(torch.Tensor, 'item', lambda self, *a, **k: self.is_cuda)
wrap(torch.Tensor, 'tolist', lambda self, *a, **k: self.is_cuda)
wrap(torch.Tensor, 'to', lambda self, *a, **k: not self.is_cuda)
_tensor = torch.tensor


def tensor(*a, **k):
    if k.get('device') is not None and str(k['device']).startswith('cuda'):
        census[('tensor', site())] += 1
    return _tensor(*a, **k)


torch.tensor = tensor
describe(t, plots=False)
torch.cuda.synchronize()
print('total', sum(census.values()))
for (name, where), c in census.most_common(40):
    print('%5d  %-7s %s' % (c, name, where))
