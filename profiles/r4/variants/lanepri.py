# lane 0's stream at the device's greatest stream priority, the other lanes
# at the least (the CP then dispatches lane 0's workgroups first)
s = open("az_engine.hip").read()
old = """      hipStream_t st;
      if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess)
        return cleanup(fail(AZ_E_HIP, "hipStreamCreate failed"));
      e->lane_streams.push_back(st);"""
assert old in s
s = s.replace(old, """      hipStream_t st;
      int p_lo = 0, p_hi = 0;
      (void)hipDeviceGetStreamPriorityRange(&p_lo, &p_hi);
      if (hipStreamCreateWithPriority(&st, hipStreamNonBlocking, l == 0 ? p_hi : p_lo) != hipSuccess)
        return cleanup(fail(AZ_E_HIP, "hipStreamCreate failed"));
      e->lane_streams.push_back(st);""")
open("az_engine.hip", "w").write(s)
