set -o pipefail
bash profiles/r06_trace.sh r06c && bash profiles/run_profiles_r06.sh r06c
