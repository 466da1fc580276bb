# the 32-sweep C2 step at the shipped 2 lanes: kernel trace + PMC passes
set -e
export T=32 LANES=2
bash tools/profile_cmd.sh r06l_step tools/lanes_probe.py
