# round 4 step v: small ChaCha20-Poly1305 batches (the wave-per-packet burst kernel, <= 4 Ki packets) on this build vs
# the build before the quad-split ChaCha and AES-HP blocks (ab/pre_quad.so), same box: the quad-split keystream in throughput terms
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
CFGS="s2n-quic_amd/libqpp.so:new ab/pre_quad.so:prequad" BENCH_ARGS="--suite chacha20poly1305 --packets 4096" ROUNDS=3 bash tools/ab.sh r04v_chacha4k && \
CFGS="s2n-quic_amd/libqpp.so:new ab/pre_quad.so:prequad" BENCH_ARGS="--packets 4096" ROUNDS=3 bash tools/ab.sh r04v_aes4k
