"""Derive collision-only MJCF scenes from the reference's mjcf/ (run here only, once).

    python tests/golden/make_scenes.py

/root/reference does not exist on the GPU box, so the planner's scenes travel as derived
data: every body (name, raw pos / orientation attributes, free joints) and every collidable
geom (contype or conaffinity non-zero) with its class defaults resolved into explicit raw
attribute strings; visual meshes, materials, textures, lights, sites, inertials and actuator
defaults are dropped.  Attribute strings are copied verbatim so both loaders see exactly the
numbers the original file holds.  tests/test_scenes.py checks, where the reference is present,
that the derived and original files give identical collidable geometry.
"""
import os
import xml.etree.ElementTree as ET

REF = "/root/reference/mjcf"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "sspp_amd", "scenes")
SCENES = {"robocrane.xml": "robocrane/robocrane.xml", "stacking.xml": "stacking.xml",
          "planner.xml": "planner.xml"}
GEOM_KEEP = ("name", "type", "size", "pos", "quat", "euler", "axisangle", "contype",
             "conaffinity", "margin")
BODY_KEEP = ("name", "pos", "quat", "euler", "axisangle")


def read_defaults(node, table, parent, top):
    name = "main" if top else node.get("class")
    table.setdefault(name, {"parent": parent, "geom": {}})
    for ch in node:
        if ch.tag == "default":
            read_defaults(ch, table, name, False)
        elif ch.tag == "geom":
            table[name]["geom"].update(ch.attrib)


def resolve(table, cls, attrs):
    chain = []
    while cls is not None:
        chain.append(cls)
        cls = table.get(cls, {}).get("parent")
    out = {}
    for c in reversed(chain):
        out.update(table.get(c, {}).get("geom", {}))
    out.update(attrs)
    return out


def convert(src, dst, title):
    root = ET.parse(src).getroot()
    table = {"main": {"parent": None, "geom": {}}}
    for d in root.findall("default"):
        read_defaults(d, table, None, True)
    out = ET.Element("mujoco", {"model": root.get("model", title)})
    comp = root.find("compiler")
    ET.SubElement(out, "compiler", {k: v for k, v in (comp.attrib if comp is not None else {}).items()
                                    if k in ("angle", "eulerseq")})
    wb_out = ET.SubElement(out, "worldbody")

    def walk(node, parent_out, childclass):
        for ch in node:
            if ch.tag == "geom":
                a = resolve(table, ch.get("class", childclass), dict(ch.attrib))
                if int(a.get("contype", "1")) == 0 and int(a.get("conaffinity", "1")) == 0:
                    continue
                ET.SubElement(parent_out, "geom", {k: a[k] for k in GEOM_KEEP if k in a})
            elif ch.tag == "body":
                b = ET.SubElement(parent_out, "body", {k: ch.get(k) for k in BODY_KEEP if ch.get(k)})
                for j in ch:
                    if j.tag == "freejoint" or (j.tag == "joint" and j.get("type") == "free"):
                        ET.SubElement(b, "freejoint", {"name": j.get("name")} if j.get("name") else {})
                walk(ch, b, ch.get("childclass", childclass))

    walk(root.find("worldbody"), wb_out, "main")
    ex = [e for c in root.findall("contact") for e in c.findall("exclude")]
    if ex:
        c_out = ET.SubElement(out, "contact")
        for e in ex:
            ET.SubElement(c_out, "exclude", {"body1": e.get("body1"), "body2": e.get("body2")})
    ET.indent(out, space="  ")
    with open(dst, "w") as f:
        f.write("<!-- Collision-only scene derived from Geryyy/sspp mjcf/%s by\n"
                "     tests/golden/make_scenes.py (bodies, free joints, collidable geoms). -->\n"
                % SCENES[title])
        f.write(ET.tostring(out, encoding="unicode"))
        f.write("\n")


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, rel in SCENES.items():
        convert(os.path.join(REF, rel), os.path.join(OUT, name), name)
        print("wrote", os.path.join(OUT, name))


if __name__ == "__main__":
    main()
