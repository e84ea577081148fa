"""Bucket balance of the partition mixer (sdp_common.h mix64) against
splitmix64's finalizer on structured and random 64-bit keys: level-1 bucket
(top 10 bits) max/mean, level-1 x level-2 cell maximum, dedup table slot (low
10 bits) max/mean.  CPU only: python3 tools/mixer_quality.py"""
import numpy as np
M=np.uint64(0xFFFFFFFFFFFFFFFF)
def splitmix(x):
    x = x ^ (x >> np.uint64(30)); x = x * np.uint64(0xBF58476D1CE4E5B9)
    x = x ^ (x >> np.uint64(27)); x = x * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))
def one(x):                  # the mixer in sdp_common.h
    x = x ^ (x >> np.uint64(32)); x = x * np.uint64(0xD6E8FEB86659FD93)
    return x ^ (x >> np.uint64(32))
def f64key(v):
    b = v.view(np.uint64)
    neg = (b >> np.uint64(63)) == 1
    return np.where(neg, ~b, b | np.uint64(1<<63))
n=1<<22
rng=np.random.default_rng(1)
sets={'seq':np.arange(n,dtype=np.uint64)^np.uint64(1<<63),
      'seq*1024':(np.arange(n,dtype=np.uint64)*np.uint64(1024))^np.uint64(1<<63),
      'f64 ints':f64key(np.arange(n,dtype=np.float64)),
      'f64 randn':f64key(rng.standard_normal(n)),
      'f64 1e9+randn':f64key(1e9+rng.standard_normal(n)),
      'f64 k/1024':f64key(np.arange(n,dtype=np.float64)/1024),
      'hi bits':(np.arange(n,dtype=np.uint64)<<np.uint64(40)),
      }
with np.errstate(over='ignore'):
  for name,k in sets.items():
    for fn in (splitmix, one):
        h=fn(k)
        b1=(h>>np.uint64(54)).astype(np.int64)              # level 1: 1024 buckets
        b2=((h>>np.uint64(44))&np.uint64(1023)).astype(np.int64)
        c1=np.bincount(b1,minlength=1024); 
        c12=np.bincount(b1*1024+b2, minlength=1<<20)
        slot=(h&np.uint64(1023)).astype(np.int64)
        cs=np.bincount(slot,minlength=1024)
        print('%-14s %-8s L1 max/mean %.3f  L1L2 max %d (mean %.1f)  slot max/mean %.3f'%(name, fn.__name__, c1.max()/c1.mean(), c12.max(), c12.mean(), cs.max()/cs.mean()))
