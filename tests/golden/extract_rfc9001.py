"""Extract the RFC 9001 Appendix A known-answer vectors that the reference holds
into tests/golden/rfc9001.json (data only: hex strings + where they came from).

Run in the build container (needs /root/reference, read-only):
    python tests/golden/extract_rfc9001.py
Sources (aws/s2n-quic 0.88.0):
  quic/s2n-quic-core/src/crypto/initial.rs   A.1-A.3 (EXAMPLE_*), header masks
  quic/s2n-quic-core/src/crypto/retry.rs     A.4 (SECRET_KEY_BYTES, NONCE_BYTES, PSEUDO_PACKET, EXPECTED_TAG)
  quic/s2n-quic-crypto/src/one_rtt.rs        A.5 secret / ku secret
  specs/www.rfc-editor.org/rfc/rfc9001.txt   A.1 key/iv/hp values, A.5 packet bytes
"""
import json
import os
import re

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def consts(path):
    src = open(os.path.join(REF, path)).read()
    out = {}
    for m in re.finditer(r"pub const (\w+): \[u8; \w+\] =\s*hex!\(\s*\"([^\"]*)\"", src):
        out[m.group(1)] = re.sub(r"\s+", "", m.group(2))
    for m in re.finditer(r"const (\w+): \[u8; \d+\] =\s*hex!\(\"([0-9a-f]+)\"\)", src):
        out.setdefault(m.group(1), m.group(2))
    return out


def rfc_value(txt, label, start):
    """Value of `label` in the RFC text after offset `start`: the first `= <hex>` that follows
    the line naming the label (values may wrap over several lines)."""
    i = txt.index("\n   " + label + " ", start)
    m = re.compile(r"=\s*([0-9a-f]{8,}(?:\s+[0-9a-f]{8,})*)").search(txt, i)
    return re.sub(r"\s+", "", m.group(1))


def main():
    ini = consts("quic/s2n-quic-core/src/crypto/initial.rs")
    ret = consts("quic/s2n-quic-core/src/crypto/retry.rs")
    one = consts("quic/s2n-quic-crypto/src/one_rtt.rs")
    rfc = open(os.path.join(REF, "specs/www.rfc-editor.org/rfc/rfc9001.txt")).read()
    a1 = rfc.index("\nA.1.  Keys")
    out = {
        "source": "aws/s2n-quic 0.88.0 constants + RFC 9001 Appendix A text (tests/golden/extract_rfc9001.py)",
        "initial_salt": ini["INITIAL_SALT"],
        "dcid": ini["EXAMPLE_DCID"],
        "client_initial_secret": ini["EXAMPLE_CLIENT_INITIAL_SECRET"],
        "server_initial_secret": ini["EXAMPLE_SERVER_INITIAL_SECRET"],
        "client": {
            "key": rfc_value(rfc, "key", rfc.index("client_initial_secret", a1)),
            "iv": rfc_value(rfc, "iv", rfc.index("client_initial_secret", a1)),
            "hp": rfc_value(rfc, "hp", rfc.index("client_initial_secret", a1)),
        },
        "server": {
            "key": rfc_value(rfc, "key", rfc.index("\n   server_initial_secret", a1)),
            "iv": rfc_value(rfc, "iv", rfc.index("\n   server_initial_secret", a1)),
            "hp": rfc_value(rfc, "hp", rfc.index("\n   server_initial_secret", a1)),
        },
        "a2": {
            "payload_prefix": ini["EXAMPLE_CLIENT_INITIAL_PAYLOAD"],
            "padded_payload_len": 1162,
            "header": ini["EXAMPLE_CLIENT_INITIAL_HEADER"],
            "pn": 2, "pn_len": 4,
            "sample": "d1b1c98dd7689fb8ec11d242b123dc9b",
            "mask": "437b9aec36",
            "protected_header": "c000000001088394c8f03e5157080000449e7b9aec34",
            "protected_packet": ini["EXAMPLE_CLIENT_INITIAL_PROTECTED_PACKET"],
        },
        "a3": {
            "payload": ini["EXAMPLE_SERVER_INITIAL_PAYLOAD"],
            "header": ini["EXAMPLE_SERVER_INITIAL_HEADER"],
            "pn": 1, "pn_len": 2,
            "sample": "2cd0991cd25b0aac406a5816b6394100",
            "mask": "2ec0d8356a",
            "protected_header": "cf000000010008f067a5502a4262b5004075c0d9",
            "protected_packet": ini["EXAMPLE_SERVER_INITIAL_PROTECTED_PACKET"],
        },
        "a4": {
            "key": ret["SECRET_KEY_BYTES"],
            "nonce": ret["NONCE_BYTES"],
            "pseudo_packet": ret["PSEUDO_PACKET"],
            "tag": ret["EXPECTED_TAG"],
            "packet": ret["PACKET"],
        },
        "a5": {
            "secret": one["SECRET"],
            "ku_secret": one["KU_SECRET"],
            "key": rfc_value(rfc, "key", rfc.index("\nA.5.  ChaCha20")),
            "iv": rfc_value(rfc, "iv", rfc.index("\nA.5.  ChaCha20")),
            "hp": rfc_value(rfc, "hp", rfc.index("\nA.5.  ChaCha20")),
            "pn": 654360564, "pn_len": 3,
            "nonce": rfc_value(rfc, "nonce", rfc.index("\nA.5.  ChaCha20")),
            "header": "4200bff4",
            "plaintext": "01",
            "ciphertext": rfc_value(rfc, "payload ciphertext", rfc.index("\nA.5.  ChaCha20")),
            "sample": rfc_value(rfc, "sample", rfc.index("\nA.5.  ChaCha20")),
            "mask": rfc_value(rfc, "mask", rfc.index("\nA.5.  ChaCha20")),
            "protected_header": "4cfe4189",
            "packet": rfc_value(rfc, "packet", rfc.index("\nA.5.  ChaCha20")),
        },
    }
    with open(os.path.join(HERE, "rfc9001.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
