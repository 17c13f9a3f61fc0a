# A/B (round 6): the cache probe with an acquire fence per fingerprint match
# (round 5) instead of one per wave
p = 'az_tree.hip'
s = open(p).read()
i = s.index('    // the fingerprint matches (inserts fill a bucket in slot order: nothing')
j = s.index('        }\n      }\n    }', i) + len('        }\n      }\n    }')
old = '''    bool stop = false;
#pragma unroll
    for (int k = 0; k < kCacheBucket; ++k) {
      const uint32_t st = w[k];
      if (stop) continue;
      if (st == kCacheEmpty) {
        stop = true;
      } else if ((st & 3u) == kCacheReady && (st >> 16) == fp) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (same_board(c.keys[base + k], b)) {
          hit = k;
          hst = st;
          stop = true;
        }
      }
    }'''
s = s[:i] + old + s[j:]
open(p, 'w').write(s)
