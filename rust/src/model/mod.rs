//! Drop-in replacement for the reference's src/model/mod.rs.
//!
//! The `Net` trait keeps its two required methods (model/mod.rs:22-28) and gains
//! one provided method, `search_trees`: the device half of `Mcts::search`.
//! Because it is provided, every `T: Net` bound in the reference (learner.rs:21,
//! learner_concurrent.rs:168, main.rs) keeps compiling as written, and
//! `Mcts<T>::search` needs no extra bound.  The Connect4, TicTacToe and chess
//! nets of this directory override it with their engines (spai_search,
//! spai_ttt_search, spai_chess_search); a net that does not fails loudly.
//!
//! `Model::predict` (model/mod.rs:36-98) and `Model::train` (:100-149) keep
//! their signatures and semantics: predict runs `forward(x, false)` (which the
//! nets here send to the device), softmax over the last axis, then each state's
//! `mask_invalid_actions`; train is the reference's minibatch Adam loop over the
//! tch graph (`forward(x, true)`).  `new_resnet` builds the same modules in the
//! same order (stem conv + BN + ReLU, then `relu(x + BN(conv(relu(BN(conv(x))))))`
//! blocks), so VarStore names and checkpoints do not change.
pub mod chess;
pub mod connect_four;
pub mod tictactoe;

use std::cmp::min;

use indicatif::ProgressBar;
use ndarray::{stack, ArrayD, Axis};
use tch::{
    kind::Kind,
    nn,
    nn::{Adam, FuncT, OptimizerConfig, SequentialT, VarStore},
    Device, IndexOp, Reduction, Tensor,
};

use crate::game::State;
use crate::mcts::{Args, Tree};

/// the per-tree result of a search: normalized root visits and (root-child id, visits)
pub type SearchResult<S> = (<S as State>::Policy, Vec<(usize, f32)>);

pub trait Net {
    type State: State;
    type Args: Default;

    fn new(vs: &nn::Path, args: Self::Args) -> Self;
    fn forward(&self, x: &Tensor, train: bool) -> (Tensor, Tensor);

    /// Mcts::search (mcts.rs:196-332) over `trees` on this net's device engine:
    /// `args.num_searches` iterations per tree, then per tree (in order) the
    /// normalized root visit policy and the [(root-child id, visits)] list; the
    /// root children are left in `tree.arena[1..]` for the caller.
    fn search_trees(&self, args: &Args, trees: &mut [&mut Tree<Self::State>]) -> Vec<SearchResult<Self::State>> {
        let _ = (args, trees);
        panic!("{}: this Net has no device search (libspai implements Connect4, TicTacToe and chess)",
               std::any::type_name::<Self>())
    }

    /// ModelTrainerWorker::train_batch (learner_concurrent.rs:72-85) on the device:
    /// one train-mode forward, the policy NLL + value MSE loss, backward and one
    /// Adam step (spai_learner_train_batch), with this net's VarStore variables
    /// overwritten by the updated parameters; returns the total loss.  None: this
    /// net has no device learner and the caller keeps its tch step
    /// (patches/device_trainer.patch makes train_batch try this first).
    fn device_train_batch(&self, states: &Tensor, policies: &Tensor, values: &Tensor) -> Option<f64> {
        let _ = (states, policies, values);
        None
    }
}

pub struct Model<T: Net> {
    pub args: Args,
    pub net: T,
}

impl<T: Net> Model<T> {
    /// Model::predict (model/mod.rs:36-98): encode, one forward(train = false),
    /// softmax, then mask_invalid_actions per state; values as returned
    pub fn predict(&self, states: &Vec<&T::State>) -> (Vec<<T::State as State>::Policy>, Vec<f32>) {
        let encodings: Vec<_> = states.iter().map(|s| s.get_encoding()).collect();
        let views: Vec<_> = encodings.iter().map(|e| e.view()).collect();
        let batch = stack(Axis(0), views.as_slice()).unwrap();
        let input = Tensor::try_from(batch).unwrap();
        let (logits, value) = self.net.forward(&input, false);
        let probs = logits.softmax(-1, Kind::Float).to_device(Device::Cpu);
        let (rows, cols) = probs.size2().unwrap();
        let probs: ArrayD<f32> = (&probs).try_into().unwrap();
        let probs = probs.into_shape((rows as usize, cols as usize)).unwrap();
        let policies = states
            .iter()
            .enumerate()
            .map(|(i, s)| s.mask_invalid_actions(probs.index_axis(Axis(0), i)).unwrap())
            .collect();
        let values = Vec::<f32>::try_from(value.to_device(Device::Cpu).contiguous().view(-1)).unwrap();
        (policies, values)
    }

    /// Model::train (model/mod.rs:100-149): a fresh Adam (lr 1e-3) over the
    /// VarStore, one random permutation of the samples, `num_epochs` passes of
    /// ceil(n / batch_size) steps of -(log_softmax(p) * pi).sum() / B + MSE(v, z)
    pub fn train(&self, states: Tensor, policies: Tensor, values: Tensor, var_store: &VarStore, args: Args,
                 pb: &ProgressBar) {
        let mut opt = Adam::default().build(var_store, 1e-3).unwrap();
        let n = states.size()[0];
        let steps = (n as f32 / self.args.batch_size as f32).ceil() as i64;
        let perm = Tensor::randperm(n, (Kind::Int64, states.device()));
        let (states, policies, values) =
            (states.index_select(0, &perm), policies.index_select(0, &perm), values.index_select(0, &perm));
        pb.reset();
        for _ in 0..args.num_epochs {
            let mut last = Tensor::new();
            for k in 0..steps {
                let lo = k * args.batch_size;
                let hi = min(lo + args.batch_size, n);
                let (p, v) = self.net.forward(&states.i(lo..hi), true);
                let nll = -(p.log_softmax(-1, Kind::Float) * policies.i(lo..hi)).sum(Kind::Float) / p.size()[0];
                let loss = nll + v.mse_loss(&values.i(lo..hi), Reduction::Mean);
                opt.backward_step(&loss);
                last = loss;
            }
            pb.set_message(format!("Loss: {:.3}", last.double_value(&[])));
            pb.inc(1);
        }
        pb.finish();
    }
}

fn conv3x3(vs: &nn::Path, ci: i64, co: i64) -> nn::Conv2D {
    nn::conv2d(vs, ci, co, 3, nn::ConvConfig { padding: 1, ..Default::default() })
}

/// relu(x + BN(conv(relu(BN(conv(x)))))) (model/mod.rs:152-165)
fn resnet_block<'a>(vs: &nn::Path, h: i64) -> FuncT<'a> {
    let body = nn::seq_t()
        .add(conv3x3(vs, h, h))
        .add(nn::batch_norm2d(vs, h, Default::default()))
        .add_fn(|x| x.relu())
        .add(conv3x3(vs, h, h))
        .add(nn::batch_norm2d(vs, h, Default::default()));
    nn::func_t(move |x, train| (x + x.apply_t(&body, train)).relu())
}

/// stem conv3x3 + BN + ReLU, then `blocks` residual blocks (model/mod.rs:167-184)
pub fn new_resnet(vs: &nn::Path, blocks: u32, in_channels: i64, h: i64) -> SequentialT {
    let mut seq = nn::seq_t()
        .add(conv3x3(vs, in_channels, h))
        .add(nn::batch_norm2d(vs, h, Default::default()))
        .add_fn(|x| x.relu());
    for _ in 0..blocks {
        seq = seq.add(resnet_block(vs, h));
    }
    seq
}

// ---------------------------------------------------------------- shared by the device nets
// The device nets keep shallow handles to every tch variable in construction
// order, which is the flat parameter order of spai_net_create /
// spai_ttt_net_create / spai_chess_net_create.

/// conv (k x k, padding) + batch_norm2d, recording weight, bias, gamma, beta,
/// running mean and running var
pub(crate) fn conv_bn_tracked(vs: &nn::Path, ci: i64, co: i64, vars: &mut Vec<Tensor>) -> (nn::Conv2D, nn::BatchNorm) {
    let conv = conv_tracked(vs, ci, co, 3, 1, vars);
    let bn = nn::batch_norm2d(vs, co, Default::default());
    vars.push(bn.ws.as_ref().unwrap().shallow_clone());
    vars.push(bn.bs.as_ref().unwrap().shallow_clone());
    vars.push(bn.running_mean.shallow_clone());
    vars.push(bn.running_var.shallow_clone());
    (conv, bn)
}

pub(crate) fn conv_tracked(vs: &nn::Path, ci: i64, co: i64, k: i64, padding: i64, vars: &mut Vec<Tensor>) -> nn::Conv2D {
    let conv = nn::conv2d(vs, ci, co, k, nn::ConvConfig { padding, ..Default::default() });
    vars.push(conv.ws.shallow_clone());
    vars.push(conv.bs.as_ref().unwrap().shallow_clone());
    conv
}

pub(crate) fn linear_tracked(vs: &nn::Path, i: i64, o: i64, vars: &mut Vec<Tensor>) -> nn::Linear {
    let l = nn::linear(vs, i, o, Default::default());
    vars.push(l.ws.shallow_clone());
    vars.push(l.bs.as_ref().unwrap().shallow_clone());
    l
}

/// new_resnet with every variable recorded (same modules, same order)
pub(crate) fn resnet_tracked(vs: &nn::Path, blocks: u32, in_channels: i64, h: i64, vars: &mut Vec<Tensor>) -> SequentialT {
    let (c, b) = conv_bn_tracked(vs, in_channels, h, vars);
    let mut seq = nn::seq_t().add(c).add(b).add_fn(|x| x.relu());
    for _ in 0..blocks {
        let (c1, b1) = conv_bn_tracked(vs, h, h, vars);
        let (c2, b2) = conv_bn_tracked(vs, h, h, vars);
        let body = nn::seq_t().add(c1).add(b1).add_fn(|x| x.relu()).add(c2).add(b2);
        seq = seq.add(nn::func_t(move |x, train| (x + x.apply_t(&body, train)).relu()));
    }
    seq
}

/// the recorded variables flattened into one f32 vector
pub(crate) fn flat_params(vars: &[Tensor]) -> Vec<f32> {
    let mut p = Vec::new();
    for t in vars {
        let v = Vec::<f32>::try_from(t.to_device(Device::Cpu).to_kind(Kind::Float).contiguous().view(-1)).unwrap();
        p.extend_from_slice(&v);
    }
    p
}

/// bit-exact fingerprint of the variables' values: FNV-1a over every f32 bit pattern in
/// construction order, so a device copy of the weights is rebuilt after any trainer ->
/// self-play copy or VarStore::load.  A NaN or infinite value panics: a diverged model is
/// reported (the reference panics on NaN too, quirk Q11) instead of every call rebuilding
/// the device copy, since a NaN fingerprint would never equal itself
pub(crate) fn fingerprint(vars: &[Tensor]) -> u64 {
    let _g = tch::no_grad_guard();
    let mut h = 0xcbf2_9ce4_8422_2325u64;
    for t in vars {
        let v = Vec::<f32>::try_from(t.to_device(Device::Cpu).to_kind(Kind::Float).contiguous().view(-1)).unwrap();
        assert!(v.iter().all(|x| x.is_finite()), "a model parameter is NaN or infinite (training diverged)");
        for x in v {
            h = (h ^ x.to_bits() as u64).wrapping_mul(0x0000_0100_0000_01b3);
        }
    }
    h
}

/// the GPU the nets' engines run on (SPAI_DEVICE, default 0)
pub(crate) fn device_index() -> i32 {
    std::env::var("SPAI_DEVICE").ok().and_then(|v| v.parse().ok()).unwrap_or(0)
}
