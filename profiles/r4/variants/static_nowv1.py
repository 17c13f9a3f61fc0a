exec(open(__file__.replace("static_nowv1.py", "static.py")).read())
exec(open(__file__.replace("static_nowv1.py", "nowv1.py")).read())
