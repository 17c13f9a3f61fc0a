# run-ahead depth 4 (az_engine.hip kRunAhead; product: 8)
s = open("az_engine.hip").read()
assert "constexpr int kRunAhead = 8;" in s
s = s.replace("constexpr int kRunAhead = 8;", "constexpr int kRunAhead = 4;")
open("az_engine.hip", "w").write(s)
