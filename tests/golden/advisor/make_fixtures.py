"""Writes the advisor fixtures: the five Prometheus query response bodies advisor.Init reads
(advisor.go:16-20, :63-147), shaped as /api/v1/query returns them, with rows that exercise
each rule of advisor.go:149-265, and expected.json, the Result.Info derived BY HAND from the Go
text (not by running yoda_amd.pack.pack_advisor).  The reference's own advisor test
(advisor_test.go:8-18) only prints a live response, so these are the build's fixtures."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def resp(rows):
    return {"status": "success", "data": {"resultType": "vector", "result": [
        {"metric": m, "value": v} for m, v in rows]}}


T = 1700000000.1
cpu = resp([
    ({"kubernetes_io_hostname": "node-a", "instance": "10.0.0.1:9100"}, [T, "50"]),
    ({"kubernetes_io_hostname": " node-b ", "instance": "10.0.0.2:9100"}, [T, "5.25"]),
    ({"kubernetes_io_hostname": "node-c", "instance": "10.0.0.3:9100"}, [T, "120"]),
    ({"kubernetes_io_hostname": "node-a", "instance": "10.0.0.9:9100"}, [T, "99"]),  # dup: first wins
    ({"kubernetes_io_hostname": "node-d", "instance": "10.0.0.4:9100"}, [T, "0"]),
])
memory = resp([
    ({"kubernetes_io_hostname": "node-a"}, [T, "31.5"]),
    ({"kubernetes_io_hostname": "node-z"}, [T, "77"]),  # no CPU entry: dropped
    ({"instance": "node-b"}, [T, "44"]),                 # no hostname, and no fallback here
])
disk = resp([
    ({"kubernetes_io_hostname": "node-a", "instance": "10.0.0.1:9100"}, [T, "10"]),
    ({"kubernetes_io_hostname": "", "instance": " node-b "}, [T, "0.5"]),  # instance fallback
    ({"instance": "node-c"}, [T, "0"]),
    ({"kubernetes_io_hostname": "node-y", "instance": "x"}, [T, "3"]),     # orphan: dropped
    ({"kubernetes_io_hostname": "node-a"}, [T, "12.5"]),                   # later row wins
    ({"kubernetes_io_hostname": "node-d"}, [T, "400"]),
])
net_up = resp([
    ({"kubernetes_io_hostname": "node-a"}, [T, "1.5"]),
    ({"kubernetes_io_hostname": "node-b"}, [T, "not-a-number"]),  # ends Init, without an error
    ({"kubernetes_io_hostname": "node-c"}, [T, "2"]),
])
net_down = resp([({"kubernetes_io_hostname": "node-a"}, [T, "9"])])

# node-a: cpu 50 (first of two), memory 31.5, disk 12.5 (the later row), up 1.5;
# node-b (trimmed): cpu 5.25, memory 0 (its memory row has no hostname), disk 0.5 (instance
#   fallback, trimmed), up 0 (its bad value ends Init before it is set);
# node-c: cpu 120, disk 0 (instance), up 0 (never reached); node-d: cpu 0, disk 400.
# NetworkIODown is never read: Init returned at node-b's network-up row.
Z = {"Memory": 0.0, "DiskIO": 0.0, "NetworkIOUp": 0.0, "NetworkIODown": 0.0}
want = {"node-a": dict(Z, Cpu=50.0, Memory=31.5, DiskIO=12.5, NetworkIOUp=1.5),
        "node-b": dict(Z, Cpu=5.25, DiskIO=0.5),
        "node-c": dict(Z, Cpu=120.0),
        "node-d": dict(Z, Cpu=0.0, DiskIO=400.0)}

if __name__ == "__main__":
    for name, d in (("cpu", cpu), ("memory", memory), ("diskio", disk), ("net_up", net_up),
                    ("net_down", net_down)):
        json.dump(d, open(os.path.join(HERE, f"{name}.json"), "w"), indent=1)
    json.dump({"info": want, "err": None}, open(os.path.join(HERE, "expected.json"), "w"),
              indent=1)
