"""Real-data ingestion: the Taylor-impact dataset format.

On-disk format (datasets/taylor_impact_2d/build_dataset.py:310-381):
  `{train,valid,test}.npz` holding one key `trajectories`, a dict
  name -> (positions[T, N, d], particle_types[N], stresses[T, N]) saved with
  `np.savez` (an object array, i.e. a pickle inside the .npy member), plus
  `metadata.json` (vel/acc/stress stats, sequence_length, file lists).

Reading.  The reference opens the file with `np.load(allow_pickle=True)`
(taylor_impact_data_loader.py:85-86), which executes whatever the pickle
names.  Here the object member is decoded by a restricted unpickler that only
resolves numpy's array/dtype/scalar reconstructors (dicts, tuples, strings and
numbers are plain pickle opcodes): a data file cannot run code.  A pickle-free
"flat" layout (`<name>/positions`, `<name>/particle_types`, `<name>/stresses`)
is read with `allow_pickle=False`; `save_trajectories` writes either.

Host API (same names, item layouts and quirks as the reference):
  TaylorImpactSamplesDataset / TaylorImpactTrajectoriesDataset / collate_fn /
  get_data_loader_by_samples / get_data_loader_by_trajectories /
  get_dataset_info (taylor_impact_data_loader.py:96-380), read_metadata
  (utils/reading_utils.py:21-31).

Device path.  `DeviceSamples` keeps every trajectory of a split resident in
HBM once ([N, T_total, d] per trajectory: even thousands of 8,000-particle
trajectories are a few GB against 288 GB) and builds each training batch by
slicing windows on the device — the same samples, in the same order (the
reference DataLoader's RandomSampler / BatchSampler), with no per-step host
collate or PCIe copy.
"""
from __future__ import annotations

import io
import json
import os
import pickle
import zipfile
from pathlib import Path
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

try:
    from numpy._core import multiarray as _multiarray
except ImportError:  # numpy < 2
    from numpy.core import multiarray as _multiarray

Trajectory = Tuple[np.ndarray, np.ndarray, np.ndarray]


# ---------------------------------------------------------------------------
# metadata (utils/reading_utils.py:21-31)
def read_metadata(data_path: str) -> dict:
    """metadata.json of a dataset directory."""
    with open(os.path.join(data_path, "metadata.json"), "rt") as fp:
        return json.loads(fp.read())


# ---------------------------------------------------------------------------
# npz reading without executing pickles
_NUMPY_GLOBALS = {
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
    ("numpy", "ndarray"), ("numpy", "dtype"),
}


class _ArrayUnpickler(pickle.Unpickler):
    """Resolves only numpy's ndarray / dtype / scalar reconstructors."""

    def find_class(self, module, name):
        if (module, name) in _NUMPY_GLOBALS:
            if name in ("_reconstruct", "scalar"):
                return getattr(_multiarray, name)
            return getattr(np, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a data file "
                                     "(only numpy arrays, dicts, tuples, strings and numbers)")


def _read_npy_member(zf: zipfile.ZipFile, member: str):
    with zf.open(member) as f:
        buf = io.BytesIO(f.read())
    version = np.lib.format.read_magic(buf)
    if version == (1, 0):
        shape, fortran, dtype = np.lib.format.read_array_header_1_0(buf)
    else:
        shape, fortran, dtype = np.lib.format.read_array_header_2_0(buf)
    if dtype.hasobject:
        return _ArrayUnpickler(buf).load()
    buf.seek(0)
    return np.lib.format.read_array(buf, allow_pickle=False)


def load_trajectories(path: str) -> Dict[str, Trajectory]:
    """name -> (positions[T,N,d], particle_types[N], stresses[T,N]) from either
    layout; raises FileNotFoundError like taylor_impact_data_loader.py:81-83."""
    p = Path(path)
    if not p.exists():
        raise FileNotFoundError(f"Data file not found: {p}")
    with zipfile.ZipFile(p) as zf:
        names = [n[:-4] for n in zf.namelist() if n.endswith(".npy")]
        if "trajectories" in names:
            obj = _read_npy_member(zf, "trajectories.npy")
            if isinstance(obj, np.ndarray) and obj.dtype == object and obj.shape == ():
                obj = obj.item()
            if not isinstance(obj, dict):
                raise ValueError(f"{p}: 'trajectories' is not a dict")
            return dict(obj)
    with np.load(p, allow_pickle=False) as z:
        out: Dict[str, Trajectory] = {}
        for key in z.files:
            if key.endswith("/positions"):
                name = key[: -len("/positions")]
                out[name] = (z[key], z[name + "/particle_types"], z[name + "/stresses"])
        if not out:
            raise ValueError(f"{p}: neither a 'trajectories' dict nor flat <name>/positions arrays")
        return out


def save_trajectories(path: str, trajectories: Dict[str, Trajectory], reference_format: bool = False) -> None:
    """Write a split; reference_format=True writes the reference's pickled dict
    (build_dataset.py:313), otherwise the pickle-free flat layout."""
    if reference_format:
        np.savez(path, trajectories=trajectories)
        return
    flat = {}
    for name, (pos, types, stress) in trajectories.items():
        flat[f"{name}/positions"] = np.asarray(pos)
        flat[f"{name}/particle_types"] = np.asarray(types)
        flat[f"{name}/stresses"] = np.asarray(stress)
    np.savez(path, **flat)


# ---------------------------------------------------------------------------
# host datasets (taylor_impact_data_loader.py:17-240)
class BaseTaylorImpactDataset:
    def _load_stress_stats_from_metadata(self, data_path: str) -> Optional[Dict]:
        """taylor_impact_data_loader.py:20-51."""
        metadata_path = Path(data_path).parent / "metadata.json"
        if not metadata_path.exists():
            return None
        try:
            with open(metadata_path) as f:
                md = json.load(f)
        except (OSError, ValueError):
            return None
        m, s = md.get("stress_mean"), md.get("stress_std")
        return {"mean": m, "std": s} if m is not None and s is not None else None

    def denormalize_stress(self, normalized_stress: np.ndarray) -> np.ndarray:
        st = getattr(self, "_stress_stats", None)
        return normalized_stress if st is None else normalized_stress * st["std"] + st["mean"]

    def _load_data(self, data_path: str) -> List[Trajectory]:
        """taylor_impact_data_loader.py:68-93 (entries that are not 3-tuples are skipped)."""
        return [t for t in load_trajectories(data_path).values() if isinstance(t, tuple) and len(t) == 3]


class TaylorImpactSamplesDataset(torch.utils.data.Dataset, BaseTaylorImpactDataset):
    """Training windows (taylor_impact_data_loader.py:96-181): sample idx maps to
    trajectory k and time_idx = T_in + (idx - start_k); the window is
    positions[time_idx - T_in : time_idx] as [N, T_in, d]."""

    def __init__(self, data_path: str, input_length_sequence: int = 6, load_stress_stats: bool = True):
        super().__init__()
        self._data = self._load_data(data_path)
        self._input_length_sequence = input_length_sequence
        if len(self._data) == 0:
            raise ValueError(f"No trajectories found in {data_path}")
        self._dimension = self._data[0][0].shape[-1]
        self._stress_stats = self._load_stress_stats_from_metadata(data_path) if load_stress_stats else None
        self._data_lengths = [x.shape[0] - input_length_sequence for x, _, _ in self._data]
        self._length = sum(self._data_lengths)
        self._cumulative_lengths = np.cumsum([0] + self._data_lengths[:-1])

    def __len__(self):
        return self._length

    def locate(self, idx: int) -> Tuple[int, int]:
        """(trajectory index, time_idx) of sample idx (:162-164)."""
        k = int(np.searchsorted(self._cumulative_lengths, idx, side="right") - 1)
        return k, int(self._input_length_sequence + (idx - self._cumulative_lengths[k]))

    def __getitem__(self, idx: int) -> Dict:
        k, t = self.locate(idx)
        positions, particle_types, stresses = self._data[k]
        win = np.transpose(positions[t - self._input_length_sequence:t], (1, 0, 2))
        # every particle gets the first particle's type (:172)
        types = np.full(win.shape[0], particle_types[0], dtype=int)
        return {"input": {"positions": win.astype(np.float32), "particle_type": types,
                          "n_particles_per_example": win.shape[0]},
                "output": {"next_position": positions[t].astype(np.float32),
                           "next_strain": stresses[t].astype(np.float32)},
                "meta": {"trajectory_idx": k, "time_idx": t}}


class TaylorImpactTrajectoriesDataset(torch.utils.data.Dataset, BaseTaylorImpactDataset):
    """Whole trajectories for rollouts (taylor_impact_data_loader.py:184-240)."""

    def __init__(self, data_path: str, load_stress_stats: bool = True):
        super().__init__()
        self._data = self._load_data(data_path)
        self._dimension = self._data[0][0].shape[-1] if self._data else 2
        self._length = len(self._data)
        self._stress_stats = self._load_stress_stats_from_metadata(data_path) if load_stress_stats else None

    def __len__(self):
        return self._length

    def __getitem__(self, idx: int) -> Dict:
        positions, particle_types, stresses = self._data[idx]
        positions = np.transpose(positions, (1, 0, 2))
        types = np.full(positions.shape[0], particle_types[0], dtype=int)
        return {"positions": torch.tensor(positions.astype(np.float32)).contiguous(),
                "particle_type": torch.tensor(types).contiguous(),
                "n_particles_per_example": torch.tensor(positions.shape[0]).contiguous(),
                "strains": torch.tensor(stresses.astype(np.float32)).contiguous(),
                "trajectory_idx": idx}


def collate_fn(batch: List[Dict]) -> Dict:
    """Concatenate the graphs of a batch (taylor_impact_data_loader.py:243-284)."""
    cat = lambda key, sub: [s[key][sub] for s in batch]
    return {"input": {"positions": torch.tensor(np.vstack(cat("input", "positions")), dtype=torch.float32),
                      "particle_type": torch.tensor(np.concatenate(cat("input", "particle_type"))),
                      "n_particles_per_example": torch.tensor(cat("input", "n_particles_per_example"))},
            "output": {"next_position": torch.tensor(np.vstack(cat("output", "next_position")),
                                                     dtype=torch.float32),
                       "next_strain": torch.tensor(np.concatenate(cat("output", "next_strain")),
                                                   dtype=torch.float32)},
            "meta": {"trajectory_idx": torch.tensor(cat("meta", "trajectory_idx")),
                     "time_idx": torch.tensor(cat("meta", "time_idx"))}}


def get_data_loader_by_samples(path: str, input_length_sequence: int = 6, batch_size: int = 2,
                               shuffle: bool = True, num_workers: int = 0, pin_memory: bool = True,
                               load_stress_stats: bool = True) -> torch.utils.data.DataLoader:
    ds = TaylorImpactSamplesDataset(path, input_length_sequence, load_stress_stats)
    return torch.utils.data.DataLoader(ds, batch_size=batch_size, shuffle=shuffle, num_workers=num_workers,
                                       pin_memory=pin_memory and torch.cuda.is_available(),
                                       collate_fn=collate_fn)


def get_data_loader_by_trajectories(path: str, num_workers: int = 0, pin_memory: bool = True,
                                    load_stress_stats: bool = True) -> torch.utils.data.DataLoader:
    ds = TaylorImpactTrajectoriesDataset(path, load_stress_stats)
    return torch.utils.data.DataLoader(ds, batch_size=None, shuffle=False, num_workers=num_workers,
                                       pin_memory=pin_memory and torch.cuda.is_available())


def get_dataset_info(data_path: str) -> Dict:
    """taylor_impact_data_loader.py:350-380."""
    trajs = load_trajectories(data_path)
    if not trajs:
        return {"num_trajectories": 0, "error": "No trajectories found"}
    first = next(iter(trajs.values()))
    if not (isinstance(first, tuple) and len(first) == 3):
        return {"num_trajectories": len(trajs), "error": "Unexpected data format"}
    positions, types, stresses = first
    return {"num_trajectories": len(trajs), "dimension": positions.shape[-1],
            "max_timesteps": positions.shape[0], "num_particles": positions.shape[1],
            "particle_types": list(np.unique(types)),
            "stress_range": [float(stresses.min()), float(stresses.max())]}


# ---------------------------------------------------------------------------
# device-resident samples
class DeviceSamples:
    """A split resident in device memory; batches are window slices taken on the
    device, identical to `collate_fn` over TaylorImpactSamplesDataset items."""

    def __init__(self, dataset: TaylorImpactSamplesDataset, device):
        self.ds = dataset
        self.device = torch.device(device)
        self.T = dataset._input_length_sequence
        # [N, T_total, d] per trajectory (the window layout), stresses [T_total, N]
        self.pos = [torch.from_numpy(np.ascontiguousarray(np.transpose(p, (1, 0, 2)).astype(np.float32)))
                    .to(self.device) for p, _, _ in dataset._data]
        self.stress = [torch.from_numpy(s.astype(np.float32)).to(self.device) for _, _, s in dataset._data]
        self.type0 = [int(t[0]) for _, t, _ in dataset._data]

    def __len__(self):
        return len(self.ds)

    def batch(self, indices: Sequence[int]) -> Dict:
        pos, nxt, strain, types, counts, tk, tt = [], [], [], [], [], [], []
        for idx in indices:
            k, t = self.ds.locate(int(idx))
            p = self.pos[k]
            pos.append(p[:, t - self.T:t])
            nxt.append(p[:, t])
            strain.append(self.stress[k][t])
            types.append(torch.full((p.shape[0],), self.type0[k], dtype=torch.int64, device=self.device))
            counts.append(p.shape[0])
            tk.append(k)
            tt.append(t)
        return {"input": {"positions": torch.cat(pos).contiguous(), "particle_type": torch.cat(types),
                          "n_particles_per_example": torch.tensor(counts)},
                "output": {"next_position": torch.cat(nxt).contiguous(), "next_strain": torch.cat(strain)},
                "meta": {"trajectory_idx": torch.tensor(tk), "time_idx": torch.tensor(tt)}}

    def count(self, indices: Sequence[int]) -> int:
        """Particles in a batch of samples (the loss-mean denominator)."""
        return sum(int(self.pos[self.ds.locate(int(i))[0]].shape[0]) for i in indices)

    def index_batches(self, batch_size: int = 2, shuffle: bool = True,
                      generator: Optional[torch.Generator] = None) -> Iterator[List[int]]:
        """One epoch of sample indices in the order torch's
        DataLoader(shuffle, batch_size) draws them."""
        sampler = (torch.utils.data.RandomSampler(range(len(self)), generator=generator) if shuffle
                   else torch.utils.data.SequentialSampler(range(len(self))))
        batches = iter(torch.utils.data.BatchSampler(sampler, batch_size, drop_last=False))
        # the DataLoader iterator draws its worker base seed before the sampler's
        # own seed (torch/utils/data/dataloader.py, _BaseDataLoaderIter)
        torch.empty((), dtype=torch.int64).random_(generator=generator)
        yield from batches

    def loader(self, batch_size: int = 2, shuffle: bool = True,
               generator: Optional[torch.Generator] = None) -> Iterator[Dict]:
        for idx in self.index_batches(batch_size, shuffle, generator):
            yield self.batch(idx)
