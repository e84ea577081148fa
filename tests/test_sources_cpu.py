"""Source checks of the HIP kernels that need no GPU.

__builtin_amdgcn_readfirstlane returns int; widened straight to 64 bits it
sign-extends, and a pointer rebuilt from two such words faulted on the GPU in
round 6 (the block-layout dedup, pass 1's candidate slots).  Every use goes
through sdp_common.h's uniform_u32 / uniform_u64 / uniform_ptr, which
zero-extend; this test keeps it that way."""

import os
import re

CSRC = os.path.join(os.path.dirname(__file__), '..', 'spark-df-profiling_amd', 'csrc')


def _sources():
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(('.hip', '.h', '.cpp')):
            yield f, open(os.path.join(CSRC, f)).read()


def test_readfirstlane_only_in_the_zero_extending_helper():
    uses = []
    for f, text in _sources():
        for i, line in enumerate(text.split('\n'), 1):
            code = line.split('//')[0]
            if '__builtin_amdgcn_readfirstlane' in code:
                uses.append((f, i, code.strip()))
    assert len(uses) == 1, uses
    f, _, code = uses[0]
    assert f == 'sdp_common.h' and code.startswith('__device__ __forceinline__ uint32_t uniform_u32(uint32_t v)')
    assert '(uint32_t)__builtin_amdgcn_readfirstlane((int)v)' in code


def test_uniform_u64_zero_extends_both_words():
    text = dict(_sources())['sdp_common.h']
    body = re.search(r'uint64_t uniform_u64\(uint64_t v\) \{(.*?)\}', text, re.S).group(1)
    assert '(uint64_t)uniform_u32((uint32_t)(v >> 32)) << 32' in body
    assert '(uint64_t)uniform_u32((uint32_t)v)' in body
