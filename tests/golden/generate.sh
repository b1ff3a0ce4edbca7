#!/bin/sh
# Regenerates tests/golden/*.json with OpenSSL (see gen_golden.c for why OpenSSL).
set -e
here=$(cd "$(dirname "$0")" && pwd)
gcc -O2 -Wall -o /tmp/qpp_gen_golden "$here/gen_golden.c" -lcrypto
/tmp/qpp_gen_golden "$here"
