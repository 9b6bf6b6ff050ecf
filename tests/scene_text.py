"""TEST INFRASTRUCTURE: scene text (the reference's scenes/*.txt format, Scene::loadMaterial/loadCamera/
loadGeom, src/scene.cpp:118-271) written from a parsed fixture under tests/golden/scenes, so tests that
exercise the product's own file parsers (kdpt_scene_load, the CLI) run where /root/reference is absent.
%.9g round-trips every float32 through the parsers' atof."""
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _f(*v):
    return " ".join(f"{x:.9g}" for x in v)


def write_scene_text(fixture: str, path: str, res=None, depth=None, iterations=None, file_name=None) -> str:
    js = json.load(open(os.path.join(GOLDEN, "scenes", f"{fixture}.json")))
    lines = []
    for i, m in enumerate(js["materials"]):
        lines += [f"MATERIAL {i}", f"RGB         {_f(*m['color'])}", f"SPECEX      {_f(m['specular_exponent'])}",
                  f"SPECRGB     {_f(*m['specular_color'])}", f"REFL        {_f(m['hasReflective'])}",
                  f"REFR        {_f(m['hasRefractive'])}", f"REFRIOR     {_f(m['indexOfRefraction'])}",
                  f"EMITTANCE   {_f(m['emittance'])}", ""]
    w, h = res or js["res"]
    lines += ["CAMERA", f"RES         {w} {h}", f"FOVY        {_f(js['fovy'])}",
              f"ITERATIONS  {iterations or js['iterations']}", f"DEPTH       {depth or js['depth']}",
              f"FILE        {file_name or fixture}", f"EYE         {_f(*js['eye'])}",
              f"LOOKAT      {_f(*js['lookAt'])}", f"UP          {_f(*js['up'])}", ""]
    for i, g in enumerate(js["geoms"]):
        t = g["trs"]
        lines += [f"OBJECT {i}", "sphere" if g["type"] == 0 else "cube", f"material {g['material']}",
                  f"TRANS       {_f(*t[0:3])}", f"ROTAT       {_f(*t[3:6])}", f"SCALE       {_f(*t[6:9])}", ""]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return path
