"""The reference's six result plots, same function names and file names
(BAR/vizualizator.py:5-133): four box plots of loss / accuracy
distributions and two line plots of the global / per-local-epoch metrics,
written to ``Graphs/`` at 16x10 in.  Uses the non-interactive Agg backend."""
from __future__ import annotations

import os
from pathlib import Path


def _plt():
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    return plt


def ensure_directory_exists(directory):
    os.makedirs(directory, exist_ok=True)


def _box(data, title, xlabel, ylabel, fname, output_folder, labels=None):
    plt = _plt()
    ensure_directory_exists(output_folder)
    fig = plt.figure(figsize=(16, 10))
    data = [d if len(d) else [float("nan")] for d in data]
    plt.boxplot(data)
    if labels is not None:
        plt.xticks(range(1, len(data) + 1), labels)
    plt.title(title)
    plt.xlabel(xlabel)
    plt.ylabel(ylabel)
    plt.grid(True)
    p = Path(output_folder) / fname
    plt.savefig(p)
    plt.close(fig)
    return str(p)


def plot_loss_distribution_by_worker(loss_data, output_folder="Graphs"):
    return _box(loss_data, "Loss Distribution by Worker", "Worker", "Loss", "loss_distribution_by_worker.png",
                output_folder, [str(i) for i in range(len(loss_data))])


def plot_loss_distribution_per_epoch(loss_data, output_folder="Graphs"):
    return _box(loss_data, "Loss Distribution per Local Epoch", "Epoch", "Loss", "loss_distribution_per_epoch.png",
                output_folder)


def plot_loss_distribution_per_epoch_global(loss_data, output_folder="Graphs"):
    return _box(loss_data, "Loss Distribution per Global Epoch", "Global Epoch", "Loss",
                "loss_distribution_per_epoch_global.png", output_folder)


def plot_accuracy_distribution_per_epoch_global(loss_data, output_folder="Graphs"):
    return _box(loss_data, "Accuracy Distribution per Global Epoch", "Global Epoch", "Accuracy (%)",
                "accuracy_distribution_per_epoch_global.png", output_folder)


def _lines(epochs, train_loss, train_accuracy, val_loss, val_accuracy, fname, output_folder, title):
    plt = _plt()
    ensure_directory_exists(output_folder)
    fig = plt.figure(figsize=(16, 10))
    xs = list(range(1, len(train_loss) + 1))
    plt.subplot(1, 2, 1)
    plt.plot(xs, train_loss, label="Train Loss")
    plt.plot(xs, val_loss, label="Validation Loss")
    plt.xlabel("Epoch")
    plt.ylabel("Loss")
    plt.title(f"{title}: Loss")
    plt.legend()
    plt.grid(True)
    plt.subplot(1, 2, 2)
    plt.plot(xs, train_accuracy, label="Train Accuracy")
    plt.plot(xs, val_accuracy, label="Validation Accuracy")
    plt.xlabel("Epoch")
    plt.ylabel("Accuracy (%)")
    plt.title(f"{title}: Accuracy")
    plt.legend()
    plt.grid(True)
    p = Path(output_folder) / fname
    plt.savefig(p)
    plt.close(fig)
    return str(p)


def plot_metrics_global(epochs, train_loss, train_accuracy, val_loss, val_accuracy, output_folder="Graphs"):
    return _lines(epochs, train_loss, train_accuracy, val_loss, val_accuracy, "training_metrics.png", output_folder,
                  "Global epochs")


def plot_metrics_total(epochs, train_loss, train_accuracy, val_loss, val_accuracy, rank, output_folder="Graphs"):
    return _lines(epochs, train_loss, train_accuracy, val_loss, val_accuracy, f"training_metrics_{rank}.png",
                  output_folder, f"Worker {rank}, local epochs")


def plot_all(histories: tuple, epochs_global: int, epochs_local: int, rank: int = 0, output_folder="Graphs"):
    """Write all six plots from train_global's 12-tuple (BAR/main.py:65-77)."""
    (awl, ael, gel, gea, gtl, gta, gvl, gva, wtl, wta, wvl, wva) = histories
    return [
        plot_metrics_global(epochs_global, gtl, gta, gvl, gva, output_folder),
        plot_metrics_total(epochs_global * epochs_local, wtl, wta, wvl, wva, rank, output_folder),
        plot_loss_distribution_by_worker(awl, output_folder),
        plot_loss_distribution_per_epoch(ael, output_folder),
        plot_loss_distribution_per_epoch_global(gel, output_folder),
        plot_accuracy_distribution_per_epoch_global(gea, output_folder),
    ]
