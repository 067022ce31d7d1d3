"""cgcnn -- the reference's model class on the MI355X-native LCN.

Drop-in for network/models_att.py of adgx/lcn-pose: same constructor
arguments (:478-506), same fit / predict / evaluate contract (:79-286), same
experiment/<dir_name>/{checkpoints/{final,best},summaries} layout (:431-433).
The TensorFlow graph + Session is replaced by liblcn.so (HIP kernels for
gfx950) through lcn_amd.native; there is no CPU compute path.

Deliberate differences from the reference:
  * dropout masks come from liblcn's counter-based generator (TF's random
    stream cannot be reproduced); rate, scaling and placement are TF's;
  * resuming from a checkpoint restores the weights AND keeps them (the
    reference re-runs the initializer after restoring, :177-180);
  * checkpoints are TensorFlow tensor bundles written without TensorFlow
    (lcn_amd.checkpoint / tf_bundle: the .index / .data files and variable
    names of tf.train.Saver, no .meta graph);
  * launched as one process per GPU (WORLD_SIZE > 1, e.g. torch.distributed.run
    train.py ...), fit trains data parallel: every rank draws the same batch
    permutation and steps its contiguous shard of each batch_size batch with
    SyncBN and an RCCL gradient all-reduce, which keeps the single-process
    arithmetic (the reference has no parallelism, :155, :210-212); predict /
    evaluate run the whole set on every rank; only rank 0 prints and writes.
"""
from __future__ import annotations

import json
import os
import re
import shutil
import time

import numpy as np

from lcn_amd import checkpoint as ckpt
from lcn_amd import dist
from lcn_amd.init import init_flat
from lcn_amd.native import Network

ROOT_PATH = os.path.join(os.path.dirname(os.path.realpath(__file__)), "..")
# device dataset slots (lcn_dataset_upload): train x / labels, validation x /
# labels (fit), predict x / labels
_SLOT_TX, _SLOT_TL, _SLOT_VX, _SLOT_VL, _SLOT_PX, _SLOT_PL = range(6)

# models_att.py:19-36 -- the skeleton edges used for the exponential mask
_EXP_EDGES = ((0, 1), (0, 7), (0, 4), (4, 5), (4, 7), (5, 6), (1, 7), (1, 2), (2, 3), (7, 11),
              (7, 8), (7, 14), (11, 12), (12, 13), (14, 15), (15, 16), (8, 9), (9, 10))


def get_exponential_matrix(verbose=True):
    """M[i, j] = 2^-d(i, j), d = hop distance on the skeleton (models_att.py:14-69)."""
    n = 17
    dist = np.full((n, n), np.inf)
    np.fill_diagonal(dist, 0)
    for u, v in _EXP_EDGES:
        dist[u, v] = dist[v, u] = 1
    for k in range(n):  # Floyd-Warshall, vectorised over (i, j)
        dist = np.minimum(dist, dist[:, k:k + 1] + dist[k:k + 1, :])
    exp_mat = 1 / (2 ** dist)
    if verbose:
        print("Distances matrix:")
        print(dist)
        print("exp_mat:")
        print(exp_mat)
    return exp_mat.astype(np.float32)


def shared_seed(net, rank):
    """A seed every rank agrees on: rank 0 draws it from its own (possibly
    user-seeded) global numpy stream, the host all-reduce hands it to the
    others (which contribute 0)."""
    seed = float(np.random.randint(0, 2 ** 31 - 1)) if rank == 0 else 0.0
    return int(net.allreduce_host([seed])[0])


def permutation_batches(n, batch_size):
    """Batch indices of fit's loop (models_att.py:193-200): a deque refilled
    with np.random.permutation(n) whenever fewer than batch_size indices
    remain, batch_size popped per step -- the same numpy draws in the same
    order, as array slices instead of per-index popleft()."""
    pending = np.empty(0, np.int64)
    head = 0
    while True:
        if pending.size - head < batch_size:
            pending = np.concatenate([pending[head:], np.random.permutation(n)])
            head = 0
            if pending.size < batch_size:  # the reference's popleft() runs dry
                raise IndexError("pop from an empty deque")
        yield pending[head:head + batch_size]
        head += batch_size


class base_model(object):
    def __init__(self):
        self.regularizers = []
        self.checkpoints = "final"
        self.writer = None
        self._loss_ema = None
        self._rank, self._world = 0, 1

    # ------------------------------------------------------------------ predict
    def predict(self, data, labels=None, sess=None):
        """Fixed-size batches, zero-padded last batch (models_att.py:79-132).

        BatchNorm uses the statistics of each (padded) batch, as the
        reference graph does.  The data go to HBM once and every batch is
        built there (lcn_predict_dataset); predictions come back float64."""
        net = self._get_session(sess)
        data = self._dense(data)
        size = data.shape[0]
        net.dataset_upload(_SLOT_PX, data)
        with self._rank_local(net):
            if labels is None:
                return net.predict_dataset(_SLOT_PX, size, self.batch_size)
            net.dataset_upload(_SLOT_PL, np.asarray(labels).reshape(size, -1))
            predictions, losses = net.predict_dataset(_SLOT_PX, size, self.batch_size,
                                                      lab_slot=_SLOT_PL)
        return predictions, self._mean_batch_loss(losses, size)

    def predict_tta(self, data, flip=False, rotate=False, translation=None, sess=None):
        """inference.py:70-110 without the host concatenation: predict the
        data plus its flipped / rotated (180 degrees) / translated copies and
        return data.undo's average (tools/data.py:269-287), float64 [N, 51]."""
        from lcn_amd.tta import augment_ops
        net = self._get_session(sess)
        data = self._dense(data)
        aug, undo, _ = augment_ops(flip=flip, rotate=rotate, translation=translation)
        net.dataset_upload(_SLOT_PX, data)
        with self._rank_local(net):
            return net.predict_dataset(_SLOT_PX, data.shape[0], self.batch_size, augment=aug,
                                       undo=undo)

    def _rank_local(self, net):
        """predict's batches are the reference's fixed batch_size batches with
        their own BN statistics (models_att.py:88-121): with several ranks every
        rank runs them whole, without exchanges, and gets the same result."""
        import contextlib

        @contextlib.contextmanager
        def ctx():
            if self._world > 1:
                net.comm_suspend(True)
            try:
                yield
            finally:
                if self._world > 1:
                    net.comm_suspend(False)
        return ctx()

    @staticmethod
    def _dense(data):
        if not isinstance(data, np.ndarray):
            data = data.toarray()  # sparse input (models_att.py:95-96)
        return data.reshape(data.shape[0], -1)

    def _mean_batch_loss(self, losses, size):
        # `loss += batch_loss` over float32 fetches, then loss * bs / size (:115, :129-130)
        loss = 0
        for l in losses:
            loss += np.float32(l)
        return loss * self.batch_size / size

    def _evaluate_resident(self, size, net):
        """evaluate() on the validation set already in HBM (fit's eval step)."""
        with self._rank_local(net):
            _, losses = net.predict_dataset(_SLOT_VX, size, self.batch_size, lab_slot=_SLOT_VL)
        loss = self._mean_batch_loss(losses, size)
        return "loss: {:.4e}".format(loss), loss

    def evaluate(self, data, labels, sess=None):
        t_process, t_wall = time.process_time(), time.time()
        predictions, loss = self.predict(data, labels, sess)
        string = "loss: {:.4e}".format(loss)
        if sess is None:
            string += "\ntime: {:.0f}s (wall {:.0f}s)".format(time.process_time() - t_process,
                                                             time.time() - t_wall)
        return string, loss

    # ---------------------------------------------------------------------- fit
    def fit(self, train_data, train_labels, val_data, val_labels, output_dir=None,
            starting_checkpoint=None):
        """Training loop of models_att.py:148-286 (one lcn_train_step per step)."""
        t_process, t_wall = time.process_time(), time.time()
        starting_step = 1
        net = self._net
        rank, world = self._rank, self._world
        lead = rank == 0          # the rank that prints and writes files
        say = print if lead else (lambda *a, **k: None)
        path = os.path.join(self._get_path("checkpoints"), "final", "model")
        best_path = os.path.join(self._get_path("checkpoints"), "best", "model")
        if starting_checkpoint is None:
            if lead:
                shutil.rmtree(self._get_path("checkpoints"), ignore_errors=True)
                os.makedirs(self._get_path("checkpoints"))
            self._initialize()
        else:
            found = None
            for fname in os.listdir(starting_checkpoint):
                m = re.search(r"model-(\d+)", fname)
                if m:
                    found = int(m.group(1))
            if found is None:
                raise FileNotFoundError(f"no model-<step> checkpoint in {starting_checkpoint}")
            starting_step = found
            say(f"Resuming from step {starting_step}")
            say(f"Restoring from checkpoint: {starting_checkpoint}")
            ema = ckpt.restore(net, ckpt.latest_checkpoint(starting_checkpoint))
            if ema is not None:
                self._loss_ema = list(ema)

        # tf.nn.dropout in the training graph only (fit feeds self.dropout,
        # :204; predict feeds 0, :102).  The masks come from liblcn's
        # counter-based generator, seeded outside numpy's global stream so the
        # batch permutations stay the reference's draws
        seed = int(os.environ.get("LCN_DROPOUT_SEED", int.from_bytes(os.urandom(8), "little")))
        if world > 1:  # one mask stream for the whole batch: rank 0's seed (53 bits survive the double)
            seed = int(net.allreduce_host([float(seed % 2 ** 53) if lead else 0.0])[0])
            # every rank draws the same batch permutations from here on
            np.random.seed(shared_seed(net, rank))
        net.set_dropout(float(self.dropout or 0.0), seed)
        shard = dist.shard_slice(self.batch_size, world, rank)
        losses = []
        # the deque of np.random.permutation() indices of :193-200, kept as an
        # array (same draws, same order); the arrays themselves live in HBM
        batches = permutation_batches(train_data.shape[0], self.batch_size)
        net.dataset_upload(_SLOT_TX, train_data)
        net.dataset_upload(_SLOT_TL, train_labels)
        net.dataset_upload(_SLOT_VX, self._dense(val_data))
        net.dataset_upload(_SLOT_VL, np.asarray(val_labels).reshape(val_data.shape[0], -1))
        num_steps = int(self.num_epochs * train_data.shape[0] / self.batch_size)
        eval_frequency = max(1, num_steps // self.num_epochs)
        say(f"Total steps to be done to complete all the epochs: {num_steps}")
        min_loss = 10000
        training_error, validation_error = [], []
        loss_average = float("nan")
        for step in range(starting_step, num_steps + 1):
            idx = next(batches)[shard]  # every rank draws the batch, steps its shard
            loss, learning_rate = net.train_step_indexed(_SLOT_TX, _SLOT_TL, idx)
            loss_average = self._update_loss_average(loss)

            if step % eval_frequency == 0:
                epoch = step * self.batch_size / train_data.shape[0]
                say("step {} / {} (epoch {:.2f} / {}):".format(step, num_steps, epoch,
                                                               self.num_epochs))
                say("  learning_rate = {:.2e}, loss_average = {:.4e}".format(learning_rate,
                                                                             loss_average))
                training_error.append([time.time(), step, float(loss_average)])
                string, loss = self._evaluate_resident(val_data.shape[0], net)
                losses.append(loss)
                say("validation {}".format(string))
                say("time: {:.0f}s (wall {:.0f}s)".format(time.process_time() - t_process,
                                                         time.time() - t_wall))
                validation_error.append([0, step, float(loss)])
                if lead:
                    self._write_summary(step, learning_rate, loss_average, loss)
                    ckpt.save(net, path, step, self._ckpt_meta(), self._loss_ema)
                if loss < min_loss:
                    min_loss = loss
                    if lead:
                        ckpt.save(net, best_path, step, self._ckpt_meta(), self._loss_ema)

        say("validation loss: trough = {:.4f}, mean = {:.2f}".format(
            min_loss, np.mean(losses[-10:]) if losses else float("nan")))
        t_step = (time.time() - t_wall) / max(num_steps, 1)
        if world > 1:
            net.allreduce_host([0.0])  # rank 0's files are complete when any rank returns
        if output_dir is not None and lead:
            os.makedirs(output_dir, exist_ok=True)
            with open(output_dir + "/training_error.json", "w") as f:
                f.write(json.dumps([training_error], indent=4))
            with open(output_dir + "/validation_error.json", "w") as f:
                f.write(json.dumps([validation_error], indent=4))
        if training_error:
            say("Final training error: ", training_error[-1])
            say("Final validation error: ", validation_error[-1])
        return losses, t_step

    # ----------------------------------------------------------------- helpers
    def _update_loss_average(self, loss):
        """tf.compat.v1.train.ExponentialMovingAverage(0.9) applied to the loss
        tensor (models_att.py:370-379): the shadow starts at 0 and, zero_debias
        being off by default, is reported as it is -- the first tens of steps
        read low, exactly as the reference's loss_average does."""
        if self._loss_ema is None:
            self._loss_ema = [0.0, 0]
        shadow, n = self._loss_ema
        shadow = 0.9 * shadow + 0.1 * float(loss)
        self._loss_ema = [shadow, n + 1]
        return shadow

    def _write_summary(self, step, lr, loss_average, val_loss):
        d = self._get_path("summaries")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "scalars.jsonl"), "a") as f:
            f.write(json.dumps({"step": step, "learning_rate": float(lr),
                                "loss/avg/total": float(loss_average),
                                "validation/loss": float(val_loss)}) + "\n")

    def get_var(self, name):
        net = self._get_session()
        for n, off, shape in net.param_layout():
            if n == name:
                return net.get_params()[off:off + int(np.prod(shape))].reshape(shape)
        raise KeyError(name)

    def _get_path(self, folder):
        path = os.path.dirname(os.path.realpath(__file__))
        return os.path.join(path, "..", "experiment", self.dir_name, folder)

    def _get_session(self, sess=None):
        """sess=None: restore the latest <checkpoints> checkpoint (models_att.py:445-463)."""
        if sess is not None:
            return sess
        filename = ckpt.latest_checkpoint(os.path.join(self._get_path("checkpoints"), self.checkpoints))
        if self._rank == 0:
            print(self._get_path("checkpoints"))
            print("restore from %s" % filename)
        if filename is None:
            raise FileNotFoundError("no checkpoint under " + self._get_path("checkpoints"))
        ckpt.restore(self._net, filename)
        return self._net


class cgcnn(base_model):
    def __init__(self, F=64, mask_type="locally_connected", init_type="ones", neighbour_matrix=None,
                 in_joints=17, out_joints=17, in_F=2, num_layers=2, residual=True, batch_norm=True,
                 max_norm=True, num_epochs=200, learning_rate=0.001, decay_type="exp",
                 decay_params=None, regularization=0.0, dropout=0, batch_size=200,
                 eval_frequency=200, dir_name="", checkpoints="final", is_training=True, knn=1):
        super().__init__()
        self.F = F
        self.mask_type = mask_type
        self.init_type = init_type
        assert neighbour_matrix.shape[0] == neighbour_matrix.shape[1]
        assert neighbour_matrix.shape[0] == in_joints
        self.neighbour_matrix = neighbour_matrix
        self.in_joints, self.out_joints = in_joints, out_joints
        self.num_layers = num_layers
        self.residual, self.batch_norm, self.max_norm = residual, batch_norm, max_norm
        self.num_epochs, self.learning_rate = num_epochs, learning_rate
        self.decay_type, self.decay_params = decay_type, decay_params
        self.regularization, self.dropout = regularization, dropout
        self.batch_size, self.eval_frequency = batch_size, eval_frequency
        self.dir_name = dir_name
        self.checkpoints = checkpoints
        self.in_F = in_F
        self.is_training = is_training
        self.knn = knn
        self.build_graph(in_joints, in_F)

    def build_graph(self, M_0, in_F):
        self.initialize_mask()
        if self.decay_type != "exp":
            raise AssertionError("not implemented lr decay types!")
        dp = self.decay_params or {"decay_steps": 32000, "decay_rate": 0.96}
        rank, world, local = dist.dist_env()
        self._rank, self._world = rank, world
        self._net = Network(F=self.F, in_F=in_F, num_layers=self.num_layers,
                            mask_type=self.mask_type, mask_matrix=self._mask_matrix,
                            residual=self.residual, batch_norm=self.batch_norm,
                            max_norm=self.max_norm, regularization=self.regularization,
                            learning_rate=self.learning_rate, decay_steps=dp["decay_steps"],
                            decay_rate=dp["decay_rate"], max_batch=self.batch_size,
                            device=local)
        if world > 1:
            # one process per GPU: RCCL communicator over the node's ranks; a
            # training step is then data parallel over each rank's shard
            if self.batch_size < world:
                raise ValueError(f"batch_size {self.batch_size} < {world} ranks")
            dist.comm_setup(self._net, rank, world)
        self._initialize()
        if rank == 0 and os.path.exists(self._get_path("summaries")):
            shutil.rmtree(self._get_path("summaries"))

    def initialize_mask(self):
        """models_att.py:534-574: LC mask = softmax(V, 0) (.) 1[N^T != 0] with V
        trainable and initialised to N^T; exponential mask = constant."""
        if "locally_connected" in self.mask_type:
            assert self.neighbour_matrix is not None
            L = np.asarray(self.neighbour_matrix).T
            assert L.shape == (self.in_joints, self.in_joints)
            if self.init_type != "same":
                raise ValueError("Unknown init_type: {}".format(self.init_type))
            self._mask_matrix = (L != 0).astype(np.float32)
        if "exponential" in self.mask_type:
            self._mask_matrix = get_exponential_matrix()

    def _initialize(self):
        # every replica starts from the same draw; LCN_INIT_SEED pins it (tests)
        if os.environ.get("LCN_INIT_SEED") is not None:
            seed = int(os.environ["LCN_INIT_SEED"])
        else:
            seed = shared_seed(self._net, self._rank) if self._world > 1 else None
        flat = init_flat(self._net.param_layout(), self._net.n_params, self.neighbour_matrix, seed=seed)
        self._net.set_params(flat)
        n = self._net.n_params
        self._net.set_optimizer_state(np.zeros(n, np.float32), np.zeros(n, np.float32), 0, 0.9, 0.999)
        self._loss_ema = None

    def _ckpt_meta(self):
        return {"F": self.F, "mask_type": self.mask_type, "num_layers": self.num_layers,
                "in_F": self.in_F, "knn": self.knn, "residual": self.residual,
                "batch_norm": self.batch_norm, "max_norm": self.max_norm,
                "regularization": self.regularization not in (0, None)}
