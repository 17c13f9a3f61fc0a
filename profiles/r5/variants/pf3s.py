# (not buildable: weights 3 k-steps ahead need 8 B buffers picked by the
# tap's parity (gen_kloop_asm.nbufs, schedule-checked); with one body per
# parity -- chess's 64-row tiles compile one skip body since round 5 -- the
# 2-block kernel still spilled 627 VGPRs)
raise SystemExit("pf3s: see the comment")
