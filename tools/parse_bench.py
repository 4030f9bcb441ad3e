import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"])
for x in d.get("secondary", []):
    print(json.dumps(x)[:240])
