# the committed tower (git HEAD) beside the working tree's other sources: the
# A/B base for an uncommitted tower change
import subprocess
src = subprocess.check_output(["git", "-C", "/root/repo", "show", "HEAD:custom-alphazero_amd/csrc/az_tower16.hip"])
open("az_tower16.hip", "wb").write(src)
