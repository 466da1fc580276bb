set -e
bash tools/profile_cmd.sh r06ae_ksp2 tools/ksp2_prof.py
bash tools/profile_cmd.sh r06ae_c2w tools/c2w_probe.py
