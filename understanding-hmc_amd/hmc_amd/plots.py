"""Host figures for GPU results: `plot_samples` and `make_movie`.

Restates the reference's matplotlib summaries so the drivers' last two calls
(`case1-script.py:66-67`) run on results produced by the HIP kernels:

  * `sample_summary`  — every number `plot_samples` draws (ranges, bins, per-dim
    mean / variance / bias, the stats box), computed once with NumPy from the
    sampler's result arrays (`q_chain`, `E_chain`, `dE_chain`, `R_q`, `n_eff_q`, …).
    Split out so that the figure's content is testable without pixels.
  * `plot_samples`    — the 3x3 panel of samplers.py:67-291 drawn from that summary.
  * `make_movie` / `make_slide` — the per-leapfrog PNG deck of samplers.py:843-924,
    from the chain-0 capture (`phi_q`, `decision_chain`) the kernels record.
  * `cov_ellipse` / `plot_cov_ellipse` — utils.py:21-71 (1σ and 2σ contours).

Plotting is host-only visualisation: nothing here touches the device, and
matplotlib is imported lazily (Agg backend when no display is configured).
"""
import os

import numpy as np
from scipy.stats import chi2, norm


def _plt():
    import matplotlib
    if not os.environ.get("DISPLAY") and matplotlib.get_backend().lower() not in ("agg", "pdf", "svg"):
        matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    # tick style of utils.py:2-8
    for ax in ("xtick", "ytick"):
        plt.rcParams[ax + ".major.size"] = 15
        plt.rcParams[ax + ".major.width"] = 1.
        plt.rcParams[ax + ".labelsize"] = 15
    return plt


def cov_ellipse(cov, q=None, nsig=None):
    """utils.py:21-52: axis lengths and rotation (degrees) of the confidence ellipse of a 2x2
    covariance, at confidence level q or nsig standard deviations."""
    if q is not None:
        level = np.asarray(q)
    elif nsig is not None:
        level = 2 * norm.cdf(nsig) - 1
    else:
        raise ValueError("One of `q` and `nsig` should be specified.")
    r2 = chi2.ppf(level, 2)
    w, v = np.linalg.eigh(np.asarray(cov, dtype=float))
    width, height = 2 * np.sqrt(w * r2)
    angle = np.degrees(np.arctan2(v[1, 0], v[0, 0]))
    return width, height, angle


def plot_cov_ellipse(ax, mus, covs, var_num1, var_num2, MoG_color="Blue", lw=2):
    """utils.py:55-71: 1σ and 2σ ellipses of each (mu, cov) projected on (var_num1, var_num2)."""
    from matplotlib.patches import Ellipse
    ij = np.ix_([var_num1, var_num2], [var_num1, var_num2])
    for mu, cov in zip(mus, covs):
        c2 = np.asarray(cov, dtype=float)[ij]
        center = (np.asarray(mu)[var_num1], np.asarray(mu)[var_num2])
        for k in (1, 2):
            w, h, ang = cov_ellipse(c2, nsig=k)
            e = Ellipse(xy=center, width=w, height=h, angle=ang, lw=lw, facecolor="none", edgecolor=MoG_color)
            ax.add_artist(e)
            e.set_clip_box(ax.bbox)
    return


def _widened(x, lo_pct=2.5, hi_pct=97.5, factor=2.5):
    """Inner 95% range of x, widened by `factor` about its centre (the reference's range rule)."""
    hi, lo = np.percentile(x, hi_pct), np.percentile(x, lo_pct)
    span = (hi - lo) * factor
    mid = (hi + lo) / 2.
    return mid - span / 2., mid + span / 2., span


def sample_summary(s, xmax=None, dx=None, q0=None, cov0=None):
    """Everything `plot_samples` (samplers.py:67-291) draws, as a dict of NumPy values.

    s: a finished sampler (HMC_sampler) with q_chain, E_chain, dE_chain, R_q, n_eff_q."""
    if s.q_chain is None:
        raise ValueError("plot_samples needs the stored q_chain (store_chain=True)")
    qc = np.asarray(s.q_chain)
    q1, q2 = qc[:, :, 0].ravel(), qc[:, :, 1].ravel()                     # :85-86 (all rows)
    E = np.asarray(s.E_chain)[:, 1:, :].ravel()
    E = E - E.mean()                                                       # :87-88
    dE = np.asarray(s.dE_chain)[:, 1:, :].ravel()                          # :89
    out = dict(q1=q1, q2=q2, E=E, dE=dE)
    if xmax is None:                                                       # :93-116
        out["q1_min"], out["q1_max"], q1_range = _widened(q1)
        out["q2_min"], out["q2_max"], q2_range = _widened(q2)
    else:                                                                  # :117-121
        out["q1_min"] = out["q2_min"] = -xmax
        out["q1_max"] = out["q2_max"] = xmax
        q1_range = q2_range = 2. * xmax
    out["dq1"], out["dq2"] = (q1_range / 100., q2_range / 100.) if dx is None else (dx, dx)   # :124-128
    out["E_min"], out["E_max"], E_range = _widened(E)                      # :191-198
    out["E_bins"] = np.arange(out["E_min"], out["E_max"], E_range / 100.)
    R = np.asarray(s.R_q)
    out["R_min"], out["R_max"], R_range = _widened(R)                      # :206-213
    out["R_bins"] = np.arange(out["R_min"], out["R_max"], R_range / 50.)
    out["R_median"], out["R_std"] = float(np.median(R)), float(np.std(R))
    # per-dimension moments over q_chain[:, 1:, :] (Q16), :223-226 and :249-252
    out["q_mean"] = np.array([np.mean(qc[:, 1:, i]) for i in range(s.D)])
    out["q_std"] = np.array([np.std(qc[:, 1:, i]) for i in range(s.D)])
    out["cov_diag"] = out["q_std"] ** 2
    if cov0 is not None:
        out["cov0_diag"] = np.diag(np.asarray(cov0, dtype=float)).copy()
        out["cov_ratio"] = out["cov_diag"] / out["cov0_diag"]
    if q0 is not None:
        out["bias"] = out["q_mean"] - np.asarray(q0, dtype=float)          # :255
    # stats box, :284-291
    n_eff = np.asarray(s.n_eff_q)
    med = float(np.median(n_eff))
    out["stats"] = dict(accept_R_warm_up=s.accept_R_warm_up, accept_R=s.accept_R, dt_total=s.dt_total,
                        N_total_steps=s.N_total_steps, N_samples=s.L_chain * s.Nchain, n_eff_median=med,
                        steps_per_es_median=s.N_total_steps / med,
                        steps_per_es_best=s.N_total_steps / float(np.max(n_eff)),
                        steps_per_es_worst=s.N_total_steps / float(np.min(n_eff)))
    return out


def plot_samples(s, title_prefix, show=False, savefig=False, xmax=None, dx=None, plot_normal=True, plot_cov=True,
                 q0=None, cov0=None):
    """samplers.py:67-291: 3x3 panel (q1-q2 scatter, marginals, E/dE, R-hat histogram, the
    estimated covariance and mean bias per dimension, stats box).  Returns the summary dict
    (the reference returns None; the extra return value is ignored by its callers)."""
    from scipy.stats import norm as _norm
    if plot_normal:
        assert (q0 is not None) and (cov0 is not None)                     # :133
        assert np.asarray(q0).size == s.D                                   # :134
    S = sample_summary(s, xmax=xmax, dx=dx, q0=q0, cov0=cov0)
    plt = _plt()
    ft, ft2, ftt = 25, 20, 30
    plt.close()
    fig, ax = plt.subplots(3, 3, figsize=(20, 20))
    q1_lim, q2_lim = [S["q1_min"], S["q1_max"]], [S["q2_min"], S["q2_max"]]
    ax[0, 0].scatter(S["q1"], S["q2"], s=2, c="black")
    if plot_cov:
        plot_cov_ellipse(ax[0, 0], [q0], [cov0], 0, 1, MoG_color="Blue", lw=2)
    ax[0, 0].set_xlabel("q1", fontsize=ft)
    ax[0, 0].set_ylabel("q2", fontsize=ft)
    ax[0, 0].axis("equal")
    ax[0, 0].set_xlim(q1_lim)
    ax[0, 0].set_ylim(q2_lim)
    ax[0, 1].hist(S["q2"], bins=np.arange(S["q2_min"], S["q2_max"], S["dq2"]), histtype="step", color="black",
                  orientation="horizontal", lw=2, label=(r"R = %.3f" % s.R_q[1]))
    ax[1, 0].hist(S["q1"], bins=np.arange(S["q1_min"], S["q1_max"], S["dq1"]), histtype="step", color="black",
                  lw=2, label=(r"R = %.3f" % s.R_q[0]))
    if plot_normal:                                                        # :132-138: scaled normal marginals
        cov0 = np.asarray(cov0, dtype=float)
        for k, (lo, hi, d) in enumerate(((S["q1_min"], S["q1_max"], S["dq1"]), (S["q2_min"], S["q2_max"], S["dq2"]))):
            g = np.arange(lo, hi, d / 10.)
            f = _norm.pdf(g, loc=q0[k], scale=np.sqrt(cov0[k, k])) * s.L_chain * d * s.Nchain
            if k == 0:
                ax[1, 0].plot(g, f, c="green", lw=3)
            else:
                ax[0, 1].plot(f, g, c="green", lw=3)
    ax[0, 1].set_ylim(q2_lim)
    ax[0, 1].set_ylabel("q2", fontsize=ft)
    ax[0, 1].legend(loc="upper right", fontsize=ft2)
    ax[1, 0].set_xlim(q1_lim)
    ax[1, 0].set_xlabel("q1", fontsize=ft)
    ax[1, 0].legend(loc="upper right", fontsize=ft2)
    ax[0, 2].hist(S["E"], bins=S["E_bins"], histtype="step", color="black", label="E", lw=2)
    ax[0, 2].hist(S["dE"], bins=S["E_bins"], histtype="step", color="red", label="dE", lw=2)
    ax[0, 2].set_xlim([S["E_min"], S["E_max"]])
    ax[0, 2].set_xlabel("Energy", fontsize=ft)
    ax[0, 2].legend(loc="upper right", fontsize=ft2)
    ax[1, 2].hist(s.R_q, bins=S["R_bins"], histtype="step", color="black", lw=2,
                  label=("R med/std: %.3f/ %.3f" % (S["R_median"], S["R_std"])))
    ax[1, 2].set_xlim([S["R_min"], S["R_max"]])
    ax[1, 2].set_xlabel("Rhat", fontsize=ft)
    ax[1, 2].legend(loc="upper right", fontsize=ft2)
    if cov0 is not None:                                                   # :218-279 need the true covariance
        c0, cd, cr = S["cov0_diag"], S["cov_diag"], S["cov_ratio"]
        x_lim = [0.9 * c0.min(), 1.1 * c0.max()]
        ax[2, 1].scatter(c0, cd, s=50, c="black", edgecolor="none")
        ax[2, 1].plot(x_lim, x_lim, c="black", lw=2, ls="--")
        ax[2, 1].set_xlim(x_lim)
        ax[2, 1].set_ylim([0.5 * cd.min(), 1.5 * cd.max()])
        ax[2, 1].set_xlabel("True cov", fontsize=ft)
        ax[2, 1].set_ylabel("Estimated cov", fontsize=ft)
        ax[2, 2].scatter(c0, cr, s=50, c="black", edgecolor="none")
        ax[2, 2].axhline(y=1, lw=2, c="black", ls="--")
        ax[2, 2].set_xlim(x_lim)
        ax[2, 2].set_ylim([0.5 * cr.min(), 1.5 * cr.max()])
        ax[2, 2].set_xlabel("True cov", fontsize=ft)
        ax[2, 2].set_ylabel("Ratio cov", fontsize=ft)
        if "bias" in S:
            b = S["bias"]
            y0, y1, _ = _widened(b, 0, 100)
            ax[2, 0].scatter(c0, b, s=50, c="black", edgecolor="none")
            ax[2, 0].axhline(y=0, c="black", ls="--", lw=2)
            ax[2, 0].set_xlim(x_lim)
            ax[2, 0].set_ylim([y0, y1])
            ax[2, 0].set_xlabel("True cov", fontsize=ft)
            ax[2, 0].set_ylabel("bias(mean)", fontsize=ft)
    st = S["stats"]
    box = ax[1, 1]
    box.scatter([0.0, 1.], [0.0, 1.], c="none")
    lines = []
    if s.warm_up_num > 0:
        lines.append((0.8, "RA before warm-up: %.3f" % st["accept_R_warm_up"]))
    lines += [(0.7, "RA after warm-up: %.3f" % st["accept_R"]),
              (0.6, "Total time: %.1f s" % st["dt_total"]),
              (0.5, "Total steps: %.2E" % st["N_total_steps"]),
              (0.4, "Ntot/eff med: %.1E/%.1E" % (st["N_samples"], st["n_eff_median"])),
              (0.3, "#steps/ES med: %.2E" % st["steps_per_es_median"]),
              (0.2, "#steps/ES best: %.2E" % st["steps_per_es_best"]),
              (0.1, "#steps/ES worst: %.2E" % st["steps_per_es_worst"])]
    for y, txt in lines:
        box.text(0.1, y, txt, fontsize=ft2)
    box.set_xlim([0, 1])
    box.set_ylim([0, 1])
    S["stats_text"] = [t for _, t in lines]
    tag = "%d\\%d\\%d\\%d\\%d" % (s.D, s.Nchain, s.Niter, s.warm_up_num, s.thin_rate)
    plt.suptitle("D/Nchain/Niter/Warm-up/Thin = " + tag, fontsize=ftt)
    if savefig:
        S["fname"] = title_prefix + "-samples-D%d-Nchain%d-Niter%d-Warm%d-Thin%d.png" % (
            s.D, s.Nchain, s.Niter, s.warm_up_num, s.thin_rate)
        plt.savefig(S["fname"], dpi=400, bbox_inches="tight")
    if show:
        plt.show()
    plt.close()
    return S


def make_slide(title_prefix, idx, phi_q, q_accepted, decision, q0=None, cov0=None, plot_cov=False, qmin=-3, qmax=3,
               dpi=200):
    """samplers.py:883-924: one frame — the accepted points so far (black), the trajectory up
    to this leapfrog (red if the iteration was accepted, else black), its last point enlarged."""
    plt = _plt()
    fig, ax = plt.subplots(1, figsize=(5, 5))
    if plot_cov:
        plot_cov_ellipse(ax, [q0], [cov0], 0, 1, MoG_color="Blue", lw=1.)
    if q_accepted.shape[0] > 0:
        ax.scatter(q_accepted[:, 0], q_accepted[:, 1], c="black", s=10, edgecolor="none")
    color = "red" if decision else "black"
    ax.scatter(phi_q[:, 0], phi_q[:, 1], s=5, edgecolor="none", c=color)
    ax.scatter(phi_q[-1:, 0], phi_q[-1:, 1], c=color, s=30, edgecolor="none")
    ax.plot(phi_q[:, 0], phi_q[:, 1], c=color, ls="--", lw=0.5)
    ax.set_xlim([qmin, qmax])
    ax.set_ylim([qmin, qmax])
    fname = "%s-slide-%d.png" % (title_prefix, idx)
    plt.savefig(fname, bbox_inches="tight", dpi=dpi)
    plt.close()
    return fname


def movie_frames(phi_q, decision_chain):
    """The frame list of make_movie (samplers.py:843-880) without drawing: one frame per point
    of every captured trajectory, as (iteration i, trajectory prefix length j+1, decision)."""
    frames = []
    for i, traj in enumerate(phi_q):
        d = int(np.asarray(decision_chain[i]).ravel()[0])
        for j in range(traj.shape[0]):
            frames.append((i, j + 1, d))
    return frames


def make_movie(s, title_prefix, q0=None, cov0=None, plot_cov=True, qmin=-3, qmax=3, dpi=200, max_frames=None):
    """samplers.py:843-880: a PNG per leapfrog point of chain 0's captured trajectories.
    The accepted-point trail is the first point of each earlier trajectory (as the reference).
    Returns the list of written file names (`max_frames` caps it; None = all)."""
    assert s.sampler_type == "Random"                                      # :850
    phi_q = getattr(s, "phi_q", None)
    if not phi_q:
        raise ValueError("make_movie needs the chain-0 capture: run gen_sample with N_save_chain0 > 0")
    starts = np.array([t[0, :] for t in phi_q]).reshape(-1, 2)
    names = []
    for idx, (i, j, d) in enumerate(movie_frames(phi_q, s.decision_chain)):
        if max_frames is not None and idx >= max_frames:
            break
        if idx % 100 == 0:
            print("Working on slide %d" % idx)
        names.append(make_slide(title_prefix, idx, phi_q[i][:j], starts[:i, :], d, q0, cov0, plot_cov, qmin=qmin,
                                qmax=qmax, dpi=dpi))
    print("Use the following command to make a movie:\nffmpeg -r 1 -start_number 0 -i %s-slide-%%d.png "
          "-vcodec mpeg4 -y %s-movie.mp4" % (title_prefix, title_prefix))
    return names
