"""Collisions and level-1 balance of the short-string hash (sdp_part.hip bh_short)
on structured string sets (hex counters, hex ids, labels, NUL-padded bytes).
CPU only: python3 tools/short_hash_quality.py"""
import numpy as np
M=(1<<64)-1
def mix64(x):
    x ^= x >> np.uint64(32); x *= np.uint64(0xD6E8FEB86659FD93); return x ^ (x >> np.uint64(32))
def bh_new(k0,k1,ln):
    l=(ln & np.uint64(31))
    lt=((l*np.uint64(0x9E3779)) << np.uint64(32)) | (l*np.uint64(0xB97F4B))
    m=k1*np.uint64(0x9E3779B97F4A7C15)
    return mix64(k0 ^ ((m << np.uint64(29)) | (m >> np.uint64(35))) ^ lt)
def words(strs):
    k0=np.zeros(len(strs),np.uint64); k1=np.zeros(len(strs),np.uint64); ln=np.zeros(len(strs),np.uint64)
    for i,s in enumerate(strs):
        b=s.ljust(16,b'\0')
        k0[i]=int.from_bytes(b[:8],'little'); k1[i]=int.from_bytes(b[8:16],'little'); ln[i]=len(s)
    return k0,k1,ln
n=1<<20
sets={'hex':[('%x'%i).encode() for i in range(n)],
      'hex16':[('%016x'%(i*2654435761 % (1<<64))).encode() for i in range(n)],
      'label_':[('label_%d'%i).encode() for i in range(n)],
      'nulpad':[(i%65536).to_bytes(2,'little')+bytes((i//65536)%16) for i in range(n)],
      }
with np.errstate(over='ignore'):
  for name,st in sets.items():
    k0,k1,ln=words(st)
    h=bh_new(k0,k1,ln)
    u=len(np.unique(h)); ref=len(set(st))
    b1=(h>>np.uint64(54)).astype(np.int64); c=np.bincount(b1,minlength=1024)
    print(name, 'distinct strings', ref, 'distinct hashes', u, 'L1 max/mean %.3f'%(c.max()/c.mean()))
