# chess8w on the compiled K loop (round 4's chess tower exactly)
exec(open(__file__.replace("chess8w_cc.py", "chess8w.py")).read())
exec(open(__file__.replace("chess8w_cc.py", "kloop_cc.py")).read())
