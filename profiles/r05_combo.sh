# beam3 utterance-major passes: PL tests + beam3 chain vs PL; then the extra bench lines (C5, --pipeline)
set -o pipefail
bash profiles/r05_b3pl.sh ${1:-r05y} || exit $?
bash profiles/r05_extra.sh ${2:-r05z}
