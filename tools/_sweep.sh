cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for nr in 1 2 3 4 6 8 15; do timeout -k 5 60 python -u tools/ce3b_micro.py 9472 34886 0 $nr 2>&1 | grep ce3b || exit 1; done
for ns in 3 5 7 10; do timeout -k 5 60 python -u tools/ce3b_micro.py 9472 34886 $ns 1 2>&1 | grep ce3b || exit 1; done
for nr in 1 2 3 4 8; do timeout -k 5 60 python -u tools/ce3_micro.py 18944 36845 0 $nr 2>&1 | grep "ce3 " || exit 1; done
for ns in 6 9 12 16; do timeout -k 5 60 python -u tools/ce3_micro.py 18944 63937 $ns 1 2>&1 | grep "ce3 " || exit 1; done
