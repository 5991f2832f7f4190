"""Fixtures for the scan-side decode (dbg_parquet_decode) — run in the build container, where
/root/reference exists; the outputs are committed (the GPU box has no reference tree).

Data files the reference's own tests hold, copied verbatim as fixtures:
  tests/data/parquet/alltypes_plain.parquet  (SNAPPY, PLAIN + RLE_DICTIONARY, BOOLEAN / INT32 /
                                              INT64 / FLOAT / DOUBLE / BYTE_ARRAY)
  tests/data/ontime_200.parquet              (SNAPPY, RLE_DICTIONARY, 109 columns, 199 rows)
Expected values, transcribed from the reference's own expected outputs:
  alltypes_plain: tests/sqllogictests/suites/stage/formats/parquet/select_parquet.test:2-11
                  (`select * from @data/parquet/alltypes_plain.parquet`, rows in file order);
  ontime_200:     tests/data/ontime_200.csv (the same 199 rows as CSV text, loaded by the
                  reference's stage tests next to the parquet file).
"""
import csv
import json
import os
import shutil

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "parquet")


def main():
    os.makedirs(OUT, exist_ok=True)
    for src, dst in [("tests/data/parquet/alltypes_plain.parquet", "alltypes_plain.parquet"),
                     ("tests/data/ontime_200.parquet", "ontime_200.parquet")]:
        shutil.copyfile(os.path.join(REF, src), os.path.join(OUT, dst))
    slt = open(os.path.join(REF, "tests/sqllogictests/suites/stage/formats/parquet/select_parquet.test")).read().splitlines()
    i = slt.index("select * from @data/parquet/alltypes_plain.parquet (pattern => '')")
    assert slt[i + 1] == "----"
    rows = []
    for line in slt[i + 2:]:
        if not line.strip():
            break
        # id bool tinyint smallint int bigint float double date_string string timestamp(date time)
        f = line.split(" ")
        rows.append(f[:10] + [" ".join(f[10:])])
    with open(os.path.join(REF, "tests/data/ontime_200.csv"), newline="") as fh:
        r = list(csv.reader(fh))
    header, body = r[0], r[1:]
    gold = {"alltypes_plain": {"source": "select_parquet.test:2-11", "columns": ["id", "bool_col", "tinyint_col", "smallint_col",
            "int_col", "bigint_col", "float_col", "double_col", "date_string_col", "string_col", "timestamp_col"], "rows": rows},
            "ontime_200": {"source": "tests/data/ontime_200.csv", "columns": header, "rows": body}}
    with open(os.path.join(HERE, "parquet_goldens.json"), "w") as fh:
        json.dump(gold, fh)
    print(len(rows), "alltypes rows;", len(body), "ontime rows x", len(header), "columns")


if __name__ == "__main__":
    main()
