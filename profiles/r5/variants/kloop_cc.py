# The tower's K loop as compiled HIP (k_loop, rounds 3-4) instead of the
# hand-scheduled assembly groups (k_loop_asm, az_kloop_asm.h): the A/B
# baseline of round 5's assembly loop.
s = open("az_tower16.hip").read()
assert s.count("#ifdef AZ_KLOOP_CC") == 1
s = "#define AZ_KLOOP_CC 1\n" + s
open("az_tower16.hip", "w").write(s)
