# (not buildable as a product form: weights 3 k-steps ahead need 8 B buffers
# picked by the tap's parity, and the 6 asm bodies that dispatch makes in the
# tap loop spilled 618 VGPRs in chess's 64-row kernel -- the generator keeps
# the form, gen_kloop_asm.nbufs, checked by tests/test_kloop_schedule_cpu.py)
raise SystemExit("pf3s: see the comment")
