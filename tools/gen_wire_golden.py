#!/usr/bin/env python3
"""Write tests/golden/frames/: Message.h frames produced by the reference's OWN encoder.

oracle/_ref/ref_wire (oracle/Makefile.ref) compiles pipeline_simulation/Message.h from /root/reference
and encodes each case below exactly as network_layer.cpp:764-766 + my_send (:6-31) would; its parser
(fromStr_toJson + fromJson, Message.h:355-569) decodes it back.  For every case this writes
  <name>.bin     the length-prefixed frame (reference bytes)
and manifest.json with the encode arguments and the reference parser's fields.  The CPU test
(tests/test_host_wire.py) checks host/wire.cpp against them: same bytes from the same arguments, same
fields from the reference's bytes.  Run in the build container (needs /root/reference):

  make -f oracle/Makefile.ref oracle/_ref/ref_wire && python tools/gen_wire_golden.py
"""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden", "frames")
REF = os.path.join(ROOT, "oracle", "_ref", "ref_wire")

# values files are written next to the frames (small), or name a committed archive fixture
VALUES = {
    "tricky.values": b"PK\x03\x04\x00\xff\n}\n,\nvalues : ,\n}" + bytes(range(256)),
    "empty.values": b"",
}
CASES = [
    # a data owner's aggregation receipt (data_owner.cpp:225-231): model part 1 of LeNet, reference-built archive
    ("receipt_lenet_mp1", ["client_id=2", "prev_node=-1", "size_=-1", "type_op=5", "model_part=1",
                           "t_start=1700000000123", "batch0=-1", "values=@GOLDEN/lenet5_c1/mp1_client0.pt"]),
    # the aggregator's reply (aggregator.cpp:96-101): Task(myid, aggregation_, myid)
    ("reply_lenet_mp3", ["client_id=-1", "prev_node=-1", "type_op=5", "model_part=3", "t_start=1700000000999",
                         "values=@GOLDEN/lenet5_c1/mp3_client0.pt"]),
    # values holding the delimiters, NUL and 0xff: the parser takes everything up to the final ",\n}"
    ("receipt_tricky_values", ["client_id=19", "prev_node=4", "size_=0", "type_op=5", "model_part=2",
                               "t_start=1", "batch0=-1", "values=@FRAMES/tricky.values"]),
    ("receipt_empty_values", ["client_id=0", "prev_node=-1", "type_op=5", "model_part=2", "t_start=0",
                              "values=@FRAMES/empty.values"]),
    # a kept-open forward activation (save_connection 1)
    ("forward_keep_open", ["save_connection=1", "client_id=7", "prev_node=3", "size_=128", "type_op=1",
                           "model_part=1", "t_start=9000000000000", "batch0=42", "values=@FRAMES/tricky.values"]),
    # the init node's refactor message to a data owner / the aggregator (data_owner.cpp:96-112)
    ("refactor_data_owner", ["type=2", "start=20", "end=3", "prev=2", "next=1", "dataset=0", "num_classes=10",
                             "model_name=0", "model_type=6", "data_owners=0,2,3", "read_table=1",
                             "rooting_table=0:10.0.0.1,1:10.0.0.2,2:10.0.0.3,3:10.0.0.4,-1:10.0.0.9"]),
    ("refactor_compute_node", ["type=1", "start=4", "end=19", "prev=-1", "next=2", "dataset=1", "num_classes=100",
                               "model_name=1", "model_type=2", "read_table=0"]),
    ("refactor_many_owners", ["type=2", "start=6", "end=1", "model_name=2", "num_classes=10", "dataset=0",
                              "data_owners=" + ",".join(str(i) for i in [0] + list(range(5, 40)))]),
]


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, data in VALUES.items():
        with open(os.path.join(OUT, name), "wb") as f:
            f.write(data)
    manifest = {"generator": "tools/gen_wire_golden.py", "encoder": "pipeline_simulation/Message.h "
                "(toJson + fromJson_toStr, int length prefix as my_send)", "cases": []}
    for name, args in CASES:
        real = [a.replace("GOLDEN", os.path.join(ROOT, "tests", "golden")).replace("FRAMES", OUT) for a in args]
        path = os.path.join(OUT, name + ".bin")
        subprocess.run([REF, "encode", "out=" + path] + real, check=True)
        fields = json.loads(subprocess.run([REF, "decode", path], check=True, capture_output=True,
                                           text=True).stdout)
        manifest["cases"].append({"name": name, "args": args, "bytes": os.path.getsize(path), "fields": fields})
        print(name, os.path.getsize(path))
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
