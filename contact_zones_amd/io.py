"""On-disk formats either side of the hot path.

Input side — the sites x features CSV and its feature-states file, read straight into the
packed layout the likelihood / sampler kernels consume (``obs`` int8 [N][F], -1 = NA), plus the
reference's own return shape for drop-in callers:
  read_features_packed        -> FeatureTable (obs int8, applicable states, names, families)
  read_features_from_csv      sbayes/util.py:345-414 (with encode_states :289-336): same tuple
  read_feature_occurrence_from_csv   sbayes/util.py:495-544 (counts files of the priors)
  read_universal_counts       sbayes/preprocessing.py:519-575
  read_inheritance_counts     sbayes/preprocessing.py:595-674
  compute_network             sbayes/preprocessing.py:113-178 + util.py:158-175 (Delaunay graph)

Output side — the Tracer-compatible result files of MCMC.save_samples (sbayes/mcmc_setup.py:
197-260), byte for byte:
  samples2file                sbayes/util.py:846-907 (collect_row_for_writing :744-843,
                              format_area_columns :66-80)

Readers use pandas' CSV parser with the reference's arguments (dtype=str, whitespace stripped),
so NA spellings and quoting follow the reference exactly; the per-feature state encoding is one
vectorised categorical lookup instead of a one-hot (N, F, S) array.
"""
import csv
import dataclasses

import numpy as np

from .packing import MAX_GROUPS, NONE

NA = -1  # obs code of a missing value

FEATURE_COLUMNS = ("x", "y", "id", "name", "family")


def _strip(df):
    """``data.applymap(normalize_str)`` (util.py:339-342, 359): strip every non-NA cell."""
    return df.apply(lambda col: col.map(lambda v: v.strip() if isinstance(v, str) else v))


@dataclasses.dataclass
class FeatureTable:
    """A features CSV in the kernels' layout.

    obs              int8 [N][F]: internal state index, -1 (packing.NA) for NA
    applicable       bool [F][S]: applicable states per feature (data.states)
    locations        float64 [N][2]
    site_ids, site_names, feature_names, family_names: external names, in file order
    state_names      per feature, the external state names in feature-states order
    fam_of_site      uint8 [N]: family index, 255 (packing.NONE) for none
    na_number        NA cells
    """
    obs: np.ndarray
    applicable: np.ndarray
    locations: np.ndarray
    site_ids: list
    site_names: list
    feature_names: list
    state_names: list
    family_names: list
    fam_of_site: np.ndarray
    na_number: int
    log: str

    @property
    def n_sites(self):
        return self.obs.shape[0]

    @property
    def n_features(self):
        return self.obs.shape[1]

    @property
    def n_states(self):
        return self.applicable.shape[1]

    @property
    def families(self):
        """bool [Fam][N] membership (the reference's ``families``, as bool)."""
        fam = np.zeros((len(self.family_names), self.n_sites), bool)
        has = self.fam_of_site != NONE
        fam[self.fam_of_site[has], np.nonzero(has)[0]] = True
        return fam

    def one_hot(self):
        """bool [N][F][S] (the reference's ``features``)."""
        from .packing import obs_to_features
        return obs_to_features(self.obs, self.n_states)


def _encode_states(data, feature_states):
    """encode_states (util.py:289-336) into obs codes: for feature f (in feature-states column
    order) the external states s_ext (non-NA entries of its column, in order) map to 0..len-1.
    Every non-NA value must be one of them (the reference's assertion)."""
    import pandas as pd
    n_states, n_features = feature_states.shape
    n_sites = data.shape[0]
    obs = np.full((n_sites, n_features), NA, np.int8)
    applicable = np.zeros((n_features, n_states), bool)
    state_names = []
    na_number = 0
    for f_idx, f_name in enumerate(feature_states.columns):
        f_states = feature_states[f_name]
        applicable[f_idx] = ~f_states.isna().to_numpy()
        s_ext = f_states.dropna().to_list()
        state_names.append(s_ext)
        f_raw = data[f_name]
        present = f_raw.notna().to_numpy()
        if len(set(s_ext)) == len(s_ext):
            codes = pd.Categorical(f_raw, categories=s_ext).codes.astype(np.int64)
        else:  # duplicate state names: dict(zip(...)) keeps the last index (util.py:318)
            ext_to_int = dict(zip(s_ext, range(len(s_ext))))
            codes = f_raw.map(ext_to_int).fillna(-1).to_numpy().astype(np.int64)
        unknown = present & (codes < 0)
        if unknown.any():
            print(set(f_raw[unknown]))
            print(s_ext)
            raise AssertionError(f"feature {f_name!r}: values {sorted(set(f_raw[unknown]))} are not "
                                 f"among its states {s_ext}")
        obs[:, f_idx] = np.where(present, codes, NA)
        na_number += int(np.count_nonzero(~present))
    return obs, applicable, state_names, na_number


def read_features_packed(file, feature_states_file) -> FeatureTable:
    """The sites / features CSV and its feature-states CSV (util.py:345-414) as a FeatureTable."""
    import pandas as pd
    data = _strip(pd.read_csv(file, dtype=str))
    try:
        cols = {c: data.pop(c) for c in FEATURE_COLUMNS}
    except KeyError:
        raise KeyError('The csv must contain columns "x", "y", "id","name", "family"')
    feature_states = _strip(pd.read_csv(feature_states_file, dtype=str))
    assert set(feature_states.columns) == set(data.columns)
    n_sites, n_features = data.shape
    locations = np.zeros((n_sites, 2))
    locations[:, 0] = [float(v) for v in cols["x"]]
    locations[:, 1] = [float(v) for v in cols["y"]]
    obs, applicable, state_names, na_number = _encode_states(data, feature_states)
    family = cols["family"]
    family_names = np.unique(family.dropna()).tolist()
    fam_of_site = np.full(n_sites, NONE, np.uint8)
    if len(family_names) > MAX_GROUPS:
        raise ValueError(f"{len(family_names)} families: at most {MAX_GROUPS} are supported")
    for i, name in enumerate(family_names):
        fam_of_site[(family == name).to_numpy()] = i
    log = f"{n_sites} sites with {n_features} features read from {file}. {na_number} NA value(s) found."
    return FeatureTable(obs=obs, applicable=applicable, locations=locations,
                        site_ids=cols["id"].to_list(), site_names=cols["name"].to_list(),
                        feature_names=feature_states.columns.to_list(), state_names=state_names,
                        family_names=family_names, fam_of_site=fam_of_site, na_number=na_number,
                        log=log)


def read_features_from_csv(file, feature_states_file):
    """Drop-in for sbayes.util.read_features_from_csv (util.py:345-414): returns (sites,
    site_names, features, feature_names, state_names, applicable_states, families,
    family_names, log) with the reference's types and shapes."""
    import pandas as pd
    tab = read_features_packed(file, feature_states_file)
    n = tab.n_sites
    names = pd.Series(tab.site_names, name="name")
    sites = {"locations": tab.locations, "id": list(range(n)), "cz": None, "names": names}
    site_names = {"external": pd.Series(tab.site_ids, name="id"), "internal": list(range(n))}
    feature_names = {"external": np.asarray(tab.feature_names, dtype=object),
                     "internal": list(range(tab.n_features))}
    state_names = {"external": tab.state_names,
                   "internal": [range(len(s)) for s in tab.state_names]}
    families = tab.families.astype(int)
    family_names = {"external": tab.family_names, "internal": list(range(len(tab.family_names)))}
    return (sites, site_names, tab.one_hot(), feature_names, state_names, tab.applicable,
            families, family_names, tab.log)


def read_feature_occurrence_from_csv(file, feature_states_file):
    """util.py:495-544: counts [F][S] (int) aligned with the feature-states file, plus the
    feature and state names."""
    import pandas as pd
    counts_raw = pd.read_csv(file, index_col="feature")
    feature_states = pd.read_csv(feature_states_file, dtype=str)
    n_states, n_features = feature_states.shape
    assert set(counts_raw.index) == set(feature_states.columns)
    counts_raw[counts_raw.isna()] = 0.
    feature_names = {"external": feature_states.columns.to_list(), "internal": list(range(n_features))}
    state_names = {"external": [[] for _ in range(n_features)], "internal": [[] for _ in range(n_features)]}
    counts = np.zeros((n_features, n_states))
    for f_idx, f_name in enumerate(feature_states.columns):
        for s_idx in range(n_states):
            s_name = feature_states[f_name][s_idx]
            if pd.isnull(s_name):
                continue
            counts[f_idx, s_idx] = counts_raw.loc[f_name, s_name]
            state_names["external"][f_idx].append(s_name)
            state_names["internal"][f_idx].append(s_idx)
    if not all(float(y).is_integer() for y in np.nditer(counts)):
        raise ValueError(f"The data in {file} must be count data.")
    return counts.astype(int), feature_names, state_names


def _check_names(file, feature_names, state_names, fn_file, sn_file):
    """The name checks of read_universal_counts / read_inheritance_counts
    (preprocessing.py:548-573, 633-672)."""
    if len(feature_names["external"]) != len(fn_file["external"]):
        raise ValueError("Different number of features in " + str(file) + " as in features.")
    for f in range(len(feature_names["external"])):
        if feature_names["external"][f] != fn_file["external"][f]:
            raise ValueError(f"The external feature {f + 1} in {file} differs from the one used in features.")
    if len(state_names["external"]) != len(sn_file["external"]):
        raise ValueError("Different number of features in " + str(file) + " as in features.")
    for f in range(len(state_names["external"])):
        if list(state_names["external"][f]) != list(sn_file["external"][f]):
            raise ValueError(f"The external category names for feature {f + 1} in {file} differ "
                             f"from those used in features.")


def _names_of(tab: FeatureTable):
    return ({"external": tab.feature_names, "internal": list(range(tab.n_features))},
            {"external": tab.state_names, "internal": [list(range(len(s))) for s in tab.state_names]})


def _counts_from(file, file_type, feature_states_file):
    if file_type == "counts_file":
        counts, fn, sn = read_feature_occurrence_from_csv(file, feature_states_file)
    else:  # 'features_file': counts of a features CSV (preprocessing.py:543-546)
        tab = read_features_packed(file, feature_states_file)
        counts = tab.one_hot().sum(axis=0)
        fn, sn = _names_of(tab)
    return counts, fn, sn


def read_universal_counts(tab: FeatureTable, file, file_type, feature_states_file):
    """preprocessing.py:519-575: counts [F][S] for the 'counts' prior on p_global, and a log."""
    counts, fn, sn = _counts_from(file, file_type, feature_states_file)
    if not all(float(y).is_integer() for y in np.nditer(counts)):
        raise ValueError(f"The data in {file} must be count data.")
    _check_names(file, *_names_of(tab), fn, sn)
    return counts.astype(int), f"{file_type} read from {file}"


def read_inheritance_counts(tab: FeatureTable, files, file_type, feature_states_file):
    """preprocessing.py:595-674: counts [Fam][F][S] for the 'counts' prior on p_families; families
    without a file keep zero counts (a uniform prior)."""
    n_states = max(len(s) for s in tab.state_names)
    counts_all = np.zeros((len(tab.family_names), tab.n_features, n_states))
    log = ""
    for fam_idx, fam_name in enumerate(tab.family_names):
        if fam_name not in files:
            log += f"No prior information for {fam_name}. Uniform prior used instead.\n"
            continue
        file = files[fam_name]
        counts, fn, sn = _counts_from(file, file_type, feature_states_file)
        counts_all[fam_idx] = counts
        log += f"Read counts for {fam_name} from {file}\n"
        if not all(float(y).is_integer() for y in np.nditer(counts)):
            raise ValueError(f"The data in {file} must be count data.")
        _check_names(file, *_names_of(tab), fn, sn)
    return counts_all.astype(int), log


def read_geo_cost_matrix(site_ids, file):
    """read_geo_cost_matrix (preprocessing.py:677-700, read_costs_from_csv util.py:417-428): the
    cost CSV (site ids as header and index) ordered by the features file's site ids, as float;
    made symmetric by averaging when it is not.  Returns (cost [N][N], log)."""
    import pandas as pd
    costs = pd.read_csv(file, dtype=str, index_col=0)
    costs.index = costs.index.astype(str)  # (numeric ids would otherwise index as integers)
    log = f"Geographical cost matrix read from {file}."
    assert set(costs.columns) == set(site_ids)
    cost = np.asarray(costs.loc[list(site_ids), list(site_ids)]).astype(float)
    if not np.allclose(cost, cost.T):
        cost = (cost + cost.T) / 2
        log += (".The cost matrix is not symmetric. It was made symmetric by averaging the original"
                " costs along the upper and lower triangle.")
    return cost, log


def compute_network(locations):
    """The Delaunay graph of the sites (util.py:158-175, qhull options "QJ Pp") as the CSR
    arrays the sampler takes (indptr, indices), and the Euclidean distance matrix
    (preprocessing.py:147-150, crs None)."""
    from scipy import spatial
    loc = np.asarray(locations, np.float64)
    delaunay = spatial.Delaunay(loc, qhull_options="QJ Pp")
    indptr, indices = delaunay.vertex_neighbor_vertices
    diff = loc[:, None] - loc
    return (np.asarray(indptr, np.int32), np.asarray(indices, np.int32),
            np.linalg.norm(diff, axis=-1))


# ---------------------------------------------------------------------------------------------
# Results files
# ---------------------------------------------------------------------------------------------
def format_area_columns(areas):
    """util.py:66-80: each area as a 0/1 string, tab separated."""
    a = np.asarray(areas).astype(bool)
    return "\t".join("".join("1" if v else "0" for v in row) for row in a)


def _fmt(v):
    """What csv.writer writes for a value: repr for floats (numpy floats included), str
    otherwise."""
    if isinstance(v, (float, np.floating)):
        return repr(float(v))
    return str(v)


def stats_columns(feature_names, state_names, family_names, n_zones, inheritance, simulated,
                  single_zones, params=True):
    """The column names of collect_row_for_writing (util.py:744-843), in order (params False: a
    chain logged without its parameters, the columns before and after the parameter block)."""
    cols = ["Sample", "posterior", "likelihood", "prior"]
    cols += [f"size_a{i}" for i in range(n_zones)]
    if not params:
        return cols + (["recall", "precision"] if simulated else [])
    for f in feature_names:
        cols += ["w_universal_" + str(f), "w_contact_" + str(f)]
        if inheritance:
            cols.append("w_inheritance_" + str(f))
    for f, st in zip(feature_names, state_names):
        cols += ["alpha_" + str(f) + "_" + str(s) for s in st]
    for a in range(n_zones):
        for f, st in zip(feature_names, state_names):
            cols += ["gamma_a" + str(a + 1) + "_" + str(f) + "_" + str(s) for s in st]
    if inheritance:
        for fam in family_names:
            for f, st in zip(feature_names, state_names):
                cols += ["beta_" + str(fam) + "_" + str(f) + "_" + str(s) for s in st]
    if simulated:
        cols += ["recall", "precision"]
    if single_zones:
        for a in range(n_zones):
            cols += [f"lh_a{a + 1}", f"prior_a{a + 1}", f"post_a{a + 1}"]
    return cols


def _ext(x):
    return x["external"] if isinstance(x, dict) else x


def collect_gt_for_writing(samples, data, config):
    """util.collect_gt_for_writing (util.py:657-738): the ground-truth row of simulated data —
    posterior / likelihood / prior, weights, alpha, gamma of every TRUE area (len(data.areas)),
    beta when the simulation had inheritance (config['simulation']['INHERITANCE']) and the single
    areas' lh / prior / posterior.  Returns (row dict, column names)."""
    feature_names = list(_ext(data.feature_names))
    state_names = [list(s) for s in _ext(data.state_names)]
    gt = {"posterior": samples["true_prior"] + samples["true_ll"], "likelihood": samples["true_ll"],
          "prior": samples["true_prior"]}
    cols = ["posterior", "likelihood", "prior"]
    tw = samples["true_weights"]
    for f, fn in enumerate(feature_names):
        names = ["w_universal_" + str(fn), "w_contact_" + str(fn)]
        if config["model"]["INHERITANCE"]:
            names.append("w_inheritance_" + str(fn))
        for c, name in enumerate(names):
            if name not in cols:
                cols.append(name)
            gt[name] = tw[f][c]
    pg = samples["true_p_global"][0]
    for f, fn in enumerate(feature_names):
        for st in range(len(state_names[f])):
            name = "alpha_" + str(fn) + "_" + str(state_names[f][st])
            if name not in cols:
                cols.append(name)
            gt[name] = pg[f][st]
    pz = samples["true_p_zones"]
    for a in range(len(data.areas)):
        for f, fn in enumerate(feature_names):
            for st in range(len(state_names[f])):
                name = "gamma_a" + str(a + 1) + "_" + str(fn) + "_" + str(state_names[f][st])
                if name not in cols:
                    cols.append(name)
                gt[name] = pz[a][f][st]
    sim_inh = config.get("simulation", {}).get("INHERITANCE", getattr(data, "p_inheritance", None) is not None)
    if sim_inh:
        pf = samples["true_p_families"]
        for fam, famn in enumerate(_ext(data.family_names)):
            for f, fn in enumerate(feature_names):
                for st in range(len(state_names[f])):
                    name = "beta_" + str(famn) + "_" + str(fn) + "_" + str(state_names[f][st])
                    if name not in cols:
                        cols.append(name)
                    gt[name] = pf[fam][f][st]
    if "true_lh_single_zones" in samples:
        for a in range(len(data.areas)):
            for key, name in (("true_lh_single_zones", f"lh_a{a + 1}"),
                              ("true_prior_single_zones", f"prior_a{a + 1}"),
                              ("true_posterior_single_zones", f"post_a{a + 1}")):
                cols.append(name)
                gt[name] = samples[key][a]
    return gt, cols


def collect_gt_areas_for_writing(samples):
    """util.collect_gt_areas_for_writing (util.py:741-742)."""
    return format_area_columns(samples["true_zones"])


def recall_precision(sample_zones, true_zones):
    """The stats file's recall and precision of one sample against the true zones (util.py:811-825):
    over the union of the zones, |sample & true| / |true| and |sample & true| / |sample| (NaN for
    an empty sample, as numpy's 0 / 0)."""
    sample_z = np.any(sample_zones, axis=0)
    true_z = np.any(true_zones, axis=0)
    inter = np.sum(np.minimum(sample_z, true_z), axis=0)
    with np.errstate(invalid="ignore", divide="ignore"):
        return inter / np.sum(true_z), inter / np.sum(sample_z, axis=0)


def samples2file(samples, data, config, paths):
    """sbayes.util.samples2file (util.py:846-907): the stats file (tab-separated, one row per
    logged sample, csv.DictWriter formatting) and the areas file (one line of area bit strings
    per sample); for simulated data (data.is_simulated) also the ground-truth stats and areas
    files (paths 'gt', 'gt_areas') and the stats file's recall / precision columns.  ``data``
    needs feature_names / state_names / family_names (reference dicts or plain lists),
    is_simulated and, simulated, areas."""
    ext = _ext
    print("Writing results to file ...")
    feature_names = list(ext(data.feature_names))
    state_names = [list(s) for s in ext(data.state_names)]
    inheritance = bool(config["model"]["INHERITANCE"])
    family_names = list(ext(data.family_names)) if inheritance else []
    simulated = bool(getattr(data, "is_simulated", False))
    if simulated and "gt" in paths:  # (written once per run: an independent chain c > 0 leaves them out)
        gt, gt_cols = collect_gt_for_writing(samples, data, config)
        with open(paths["gt"], "w", newline="") as fh:
            writer = csv.writer(fh, delimiter="\t")
            writer.writerow(gt_cols)
            writer.writerow([_fmt(gt[c]) for c in gt_cols])
        with open(paths["gt_areas"], "w", newline="") as fh:
            fh.write(collect_gt_areas_for_writing(samples))
    zones = samples["sample_zones"]
    n = len(zones)
    steps_per_sample = float(config["mcmc"]["N_STEPS"] / config["mcmc"]["N_SAMPLES"])
    n_zones = int(config["model"]["N_AREAS"])
    single = "sample_lh_single_zones" in samples
    # a chain logged without its parameters (an independent chain c > 0, mcmc.ChainLog): the
    # sample, posterior, likelihood, prior and size columns (and recall / precision) only
    params = "sample_weights" in samples
    cols = stats_columns(feature_names, state_names, family_names, n_zones, inheritance, simulated,
                         single, params)
    n_f = len(feature_names)
    st_idx = [list(range(len(s))) for s in state_names]
    with open(paths["parameters"], "w", newline="") as fh:
        writer = csv.writer(fh, delimiter="\t")
        for s in range(n):
            if s == 0:
                writer.writerow(cols)
            lik = samples["sample_likelihood"][s]
            pri = samples["sample_prior"][s]
            row = [str(int(s * steps_per_sample)), _fmt(pri + lik), _fmt(lik), _fmt(pri)]
            z = np.asarray(zones[s])
            row += [str(int(np.count_nonzero(a))) for a in z]
            if not params:
                if simulated:
                    row += [_fmt(v) for v in recall_precision(z, samples["true_zones"])]
                writer.writerow(row)
                continue
            w = samples["sample_weights"][s]
            for f in range(n_f):
                row += [_fmt(w[f][0]), _fmt(w[f][1])]
                if inheritance:
                    row.append(_fmt(w[f][2]))
            pg = samples["sample_p_global"][s][0]
            for f in range(n_f):
                row += [_fmt(pg[f][i]) for i in st_idx[f]]
            pz = samples["sample_p_zones"][s]
            for a in range(n_zones):
                for f in range(n_f):
                    row += [_fmt(pz[a][f][i]) for i in st_idx[f]]
            if inheritance:
                pf = samples["sample_p_families"][s]
                for fam in range(len(family_names)):
                    for f in range(n_f):
                        row += [_fmt(pf[fam][f][i]) for i in st_idx[f]]
            if simulated:
                row += [_fmt(v) for v in recall_precision(z, samples["true_zones"])]
            if single:
                for a in range(n_zones):
                    row += [_fmt(samples["sample_lh_single_zones"][s][a]),
                            _fmt(samples["sample_prior_single_zones"][s][a]),
                            _fmt(samples["sample_posterior_single_zones"][s][a])]
            writer.writerow(row)
    with open(paths["areas"], "w", newline="") as fh:
        for s in range(n):
            fh.write(format_area_columns(zones[s]) + "\n")


__all__ = ["FeatureTable", "read_features_packed", "read_features_from_csv",
           "read_feature_occurrence_from_csv", "read_universal_counts", "read_inheritance_counts",
           "compute_network", "read_geo_cost_matrix", "format_area_columns", "stats_columns", "samples2file",
           "collect_gt_for_writing", "collect_gt_areas_for_writing", "recall_precision",
           "extract_feature_states"]


def extract_feature_states(input_paths, output_path=None, order_states=True):
    """sbayes/tools/extract_feature_states.py:43-133 without the GUI: the union of the states each
    feature takes over the input CSVs (metadata columns id, name, family, x, y dropped, values
    stripped), sorted (ORDER_STATES), as the feature-states CSV (one column per feature, padded
    with empty cells).  Returns the DataFrame; writes it when ``output_path`` is given."""
    import pandas as pd
    meta = ["id", "name", "family", "x", "y"]
    states = None
    for path in input_paths:
        df = pd.read_csv(path, sep=",", dtype=str)
        for column in meta:
            if column not in df.columns:
                raise ValueError(f"Required column '{column}' missing in file {path}.")
        df = _strip(df.drop(meta, axis=1))
        new = {f: set(df[f].dropna().unique()) for f in df.columns}
        if states is None:
            states = new
        else:
            if set(states) != set(new):
                raise ValueError("\nFeatures do not match between the different input files:"
                                 f"\n\tPreviously loaded features: \t {sorted(states)}"
                                 f"\n\tFeatures in {path}: \t {sorted(new)}")
            for f in states:
                states[f].update(new[f])
    cols = {f: (sorted(v) if order_states else list(v)) for f, v in states.items()}
    n_rows = max(len(v) for v in cols.values())
    out = pd.DataFrame({f: v + [None] * (n_rows - len(v)) for f, v in cols.items()})
    if output_path is not None:
        out.to_csv(output_path, index=False, lineterminator="\n")
    return out
