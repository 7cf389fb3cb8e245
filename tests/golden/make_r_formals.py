"""Extract the formals (argument names and default expressions) of the reference's R functions
that form the drop-in surface into tests/golden/r_formals.json.

Run here, where /root/reference exists: `python tests/golden/make_r_formals.py`.  The fixture
holds only names and default expressions (the API contract), per reference script."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from rformals import parse_formals  # noqa: E402

REF = "/root/reference"
SURFACE = {
    "vert-cor.R": ["mixquant", "gen_gaussian", "gen_bernoulli", "rLap", "correlation_INT_signflip",
                   "ci_NI_signbatch", "ci_INT_signflip", "priv_standardize", "run_sim_one"],
    "ver-cor-subG.R": ["lambda_n", "lambda_INT_n", "mixquant", "correlation_NI_subG", "ci_INT_subG",
                       "gen_mix_gaussian", "gen_bounded_factor", "run_sim_one"],
    "real-data-sims.R": ["rLap", "dp_mean", "dp_sd", "standardize_dp", "standardize_age_bmi",
                         "lambda_from_priv", "lambda_n", "correlation_NI_subG", "lambda_INT_n",
                         "mixquant", "lambda_receiver_from_noise", "ci_INT_subG"],
}


def extract(ref=REF):
    out = {}
    for script, names in SURFACE.items():
        with open(os.path.join(ref, script), encoding="utf-8") as f:
            fm = parse_formals(f.read())
        out[script] = {n: fm[n] for n in names}
    return out


if __name__ == "__main__":
    data = extract()
    lines = ["{"]
    for i, (script, fns) in enumerate(data.items()):
        lines.append(f" {json.dumps(script)}: {{")
        items = list(fns.items())
        for j, (name, args) in enumerate(items):
            sep = "," if j + 1 < len(items) else ""
            lines.append(f"  {json.dumps(name)}: {json.dumps(args, ensure_ascii=False)}{sep}")
        lines.append(" }" + ("," if i + 1 < len(data) else ""))
    lines.append("}")
    with open(os.path.join(HERE, "r_formals.json"), "w", encoding="utf-8") as f:
        f.write("\n".join(lines) + "\n")
