for n in d22 d33 d44 d32 d24 d43; do C2DSR_LIB_DIR=variants/ce3_$n timeout -k 5 60 python -u tools/ce3_micro.py 2>&1 | grep ce3 | sed "s/^/$n /"; done
