"""Writes tests/golden/zparameters_reference.json: every `key = value;` of the reference's own parameter files
(FriedLiver/zParametersDefault.txt, FriedLiver/zParametersBundlingDefault.txt), read here with an independent
parser of mLib's ParameterFile format (one `name = value;` per line, `//` comments). The JSON holds the raw value
text per key, in file order: the data the two files give the boundary, so tests off this container (where
/root/reference does not exist) can rebuild parameter files with exactly these settings.
Usage: python tests/golden/make_zparameters_fixture.py [/root/reference]"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
FILES = ("zParametersDefault.txt", "zParametersBundlingDefault.txt")


def read_parameter_text(text: str) -> dict:
    """name -> raw value text (comments removed, up to the ';'), in file order; a later line wins."""
    out = {}
    for line in text.splitlines():
        line = line.split("//", 1)[0].strip()
        if "=" not in line:
            continue
        name, value = line.split("=", 1)
        value = value.split(";", 1)[0].strip()
        out[name.strip()] = value
    return out


def main(ref="/root/reference"):
    data = {"source": "kanster/BundleFusion FriedLiver/zParameters*.txt, parsed by tests/golden/make_zparameters_fixture.py"}
    for f in FILES:
        with open(os.path.join(ref, "FriedLiver", f), encoding="latin-1") as fh:
            data[f] = read_parameter_text(fh.read())
    with open(os.path.join(HERE, "zparameters_reference.json"), "w") as fh:
        json.dump(data, fh, indent=1)
    print({f: len(data[f]) for f in FILES})


if __name__ == "__main__":
    main(*sys.argv[1:])
