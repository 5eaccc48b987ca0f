"""Synthetic workloads of BASELINE.md / SURVEY.md 8(d) (splitmix64 RNG, T0 = 1_700_000_000_000 ms).

C1  every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec      (1 stream, no partition)
C2  C1 inside `partition with (symbol of StockStream)`                                  (10k keys, 1 GPU)
C3  partition with (key of S): every e1=S[price>20], e2=S[price>e1.price]<2:5>, e3=S[price<e2[last].price]
C4  partition with (key of A..D): e1=A[v>10] -> (e2=B[v>20] and e3=C[v>30]) -> not D[v>40] for 5 sec
Prices are rint((10 + 20u) * 100) / 100, u uniform in [0, 1).
"""
import numpy as np

T0 = 1_700_000_000_000
GOLDEN = np.uint64(0x9E3779B97F4A7C15)

STOCK_STREAM = "define stream StockStream (id long, symbol string, price double, volume int);"

C1_APP = ("@app:playback " + STOCK_STREAM +
          " @info(name = 'query1') from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] "
          "within 1 sec select e1.id as e1id, e2.id as e2id insert into M;")

C2_APP = ("@app:playback " + STOCK_STREAM +
          " partition with (symbol of StockStream) begin @info(name = 'query1') "
          "from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
          "select e1.id as e1id, e2.id as e2id insert into M; end;")

C3_APP = ("@app:playback define stream S (id long, key long, price double, volume int); "
          "partition with (key of S) begin @info(name = 'query1') "
          "from every e1=S[price>20], e2=S[price>e1.price]<2:5>, e3=S[price<e2[last].price] "
          "select e1.id as e1id, e2[0].id as e2f, e2[last].id as e2l, e3.id as e3id insert into M; end;")


def splitmix64(seed, n, offset=0):
    """n outputs of the splitmix64 sequence seeded with `seed` (state_i = seed + (i+1)*golden)."""
    with np.errstate(over="ignore"):
        i = np.arange(offset + 1, offset + n + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform01(z):
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def prices(seed, n, offset=0):
    u = uniform01(splitmix64(seed, n, offset))
    return np.rint((10.0 + 20.0 * u) * 100.0) / 100.0


def c1_columns(n, seed=42, adversarial=False):
    """ts, id, price, volume for C1 (ts = T0 + i)."""
    i = np.arange(n, dtype=np.int64)
    ts = T0 + i
    if adversarial:
        price = 40.0 - 0.01 * (i % 2000)
    else:
        price = prices(seed, n)
    return {"ts": ts, "id": i, "price": price, "volume": (i % 1000).astype(np.int32)}


def c2_columns(n, keys=10_000, seed=7, per_ms=100, offset=0):
    """ts, id, key index, price, volume for C2 (ts = T0 + floor(i / per_ms))."""
    i = np.arange(offset, offset + n, dtype=np.int64)
    ts = T0 + i // per_ms
    z = splitmix64(seed, n, offset)
    key = (z % np.uint64(keys)).astype(np.int64)
    price = prices(seed + 1, n, offset)
    return {"ts": ts, "id": i, "key": key, "price": price, "volume": (i % 1000).astype(np.int32)}


def symbols(keys):
    return ["S%05d" % k for k in range(keys)]


def c3_columns(keys, per_key=100, seed=11):
    n = keys * per_key
    i = np.arange(n, dtype=np.int64)
    ts = T0 + i // 10_000
    z = splitmix64(seed, n)
    key = (z % np.uint64(keys)).astype(np.int64)
    price = prices(seed + 1, n)
    return {"ts": ts, "id": i, "key": key, "price": price, "volume": (i % 1000).astype(np.int32)}


C4_STREAMS = ("A", "B", "C", "D")
C4_APP = ("@app:playback " + " ".join("define stream %s (id long, key long, v double);" % s for s in C4_STREAMS) +
          " partition with (key of A, key of B, key of C, key of D) begin @info(name = 'query1') "
          "from e1=A[v>10] -> (e2=B[v>20] and e3=C[v>30]) -> not D[v>40] for 5 sec "
          "select e1.id as e1id, e2.id as e2id, e3.id as e3id insert into M; end;")


def c4_columns(keys, per_key=20, seed=13, per_tick=10_000):
    """C4: streams A, B, C, D round-robin by global ts, keys uniform, ts = T0 + 10 floor(i / 10^4)
    so the 5 s timers fall due mid-run; v = rint(50 u * 100) / 100 in [0, 50) so every filter (v > 10 / 20 / 30 / 40)
    passes part of the events. The run ends with advance_time(ts[-1] + 5000)."""
    n = keys * per_key
    i = np.arange(n, dtype=np.int64)
    ts = T0 + 10 * (i // per_tick)
    z = splitmix64(seed, n)
    key = (z % np.uint64(keys)).astype(np.int64)
    v = np.rint(50.0 * uniform01(splitmix64(seed + 1, n)) * 100.0) / 100.0
    return {"ts": ts, "id": i, "key": key, "v": v, "stream": (i % 4).astype(np.int32)}
