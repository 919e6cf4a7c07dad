// Shared UI components (datax-common/src/components: pageHeader, panelHeader, verticalTabs, statementBox,
// topNav*, plus the Fabric controls the packages use: text fields, dropdowns, toggles, message bars, dialogs).
import { h, mount } from './dom.js';

// ---- user context (datax-common modules/user + functionEnabled) -----------------------------------------------
export const userContext = {
    user: { name: '', roles: [], isWriter: false },
    functions: {},
    enableLocalOneBox: false
};

export function functionEnabled(name) {
    return !!userContext.functions[name];
}

// ---- layout ------------------------------------------------------------------------------------------------------
export function PageHeader(title, ...actions) {
    return h('div', { class: 'page-header' }, h('h2', null, title), h('div', { class: 'actions' }, actions));
}

export function PanelHeader(title, ...extra) {
    return h('div', { class: 'panel-header' }, h('span', null, title), extra);
}

export function StatementBox(icon, text) {
    return h('div', { class: 'statement' }, h('span', { class: 'icon' }, icon || 'i'), h('span', null, text));
}

// Vertical tabs with a validity marker per tab (verticalTabs.jsx: a red marker on tabs whose content is invalid)
export function VerticalTabs(tabs, selected, onSelect) {
    const nav = h(
        'div',
        { class: 'vtabs-nav' },
        tabs.map(t =>
            h(
                'button',
                {
                    class: 'vtab' + (t.key === selected ? ' on' : '') + (t.valid === false ? ' invalid' : ''),
                    'data-tab': t.key,
                    onclick: () => onSelect(t.key)
                },
                t.label,
                t.valid === false ? h('span', { class: 'marker', title: 'incomplete settings' }, ' ●') : null
            )
        )
    );
    const cur = tabs.find(t => t.key === selected) || tabs[0];
    const body = h('div', { class: 'vtabs-body' }, cur ? cur.render() : null);
    return h('div', { class: 'vtabs' }, nav, body);
}

// ---- messages ----------------------------------------------------------------------------------------------------
export function MessageBar(kind, text, onDismiss) {
    if (!text) return null;
    return h(
        'div',
        { class: 'msgbar ' + (kind || 'info') },
        h('span', null, text),
        onDismiss ? h('button', { class: 'link', onclick: onDismiss }, '✕') : null
    );
}

export function Spinner(label) {
    return h('div', { class: 'spinner' }, h('span', { class: 'spin' }), label || 'Loading...');
}

export function confirmDialog(title, text) {
    return new Promise(resolve => {
        const close = v => {
            document.body.removeChild(overlay);
            resolve(v);
        };
        const overlay = h(
            'div',
            { class: 'overlay' },
            h(
                'div',
                { class: 'dialog', role: 'dialog' },
                h('h3', null, title),
                h('p', null, text),
                h(
                    'div',
                    { class: 'actions' },
                    h('button', { class: 'primary', onclick: () => close(true) }, 'Yes'),
                    h('button', { onclick: () => close(false) }, 'No')
                )
            )
        );
        document.body.appendChild(overlay);
    });
}

// ---- form controls -----------------------------------------------------------------------------------------------
// every control takes (label, value, onChange, opts) and returns a labelled row; opts.disabled gates writers
export function TextField(label, value, onChange, opts) {
    opts = opts || {};
    const input = h(opts.multiline ? 'textarea' : 'input', {
        class: opts.mono ? 'mono' : null,
        value: value === undefined || value === null ? '' : String(value),
        placeholder: opts.placeholder,
        disabled: opts.disabled,
        spellcheck: opts.multiline ? 'false' : null,
        style: opts.height ? { height: opts.height } : null,
        type: opts.type,
        oninput: e => onChange(e.target.value)
    });
    const err = opts.validate ? opts.validate(value) : null;
    return h(
        'label',
        { class: 'field' + (err ? ' error' : '') },
        h('span', { class: 'label' }, label),
        input,
        err ? h('span', { class: 'errtext' }, err) : null
    );
}

export function Dropdown(label, options, value, onChange, opts) {
    opts = opts || {};
    const sel = h(
        'select',
        { disabled: opts.disabled, onchange: e => onChange(e.target.value) },
        options.map(o =>
            h('option', { value: o.key, selected: o.key === value ? true : null, disabled: o.disabled }, o.name)
        )
    );
    return h('label', { class: 'field' }, h('span', { class: 'label' }, label), sel);
}

export function Toggle(label, value, onChange, opts) {
    opts = opts || {};
    return h(
        'label',
        { class: 'field toggle' },
        h('input', { type: 'checkbox', checked: !!value, disabled: opts.disabled, onchange: e => onChange(e.target.checked) }),
        h('span', { class: 'label' }, label)
    );
}

export function Slider(label, value, min, max, onChange, opts) {
    opts = opts || {};
    const out = h('span', { class: 'slider-value' }, String(value));
    return h(
        'label',
        { class: 'field' },
        h('span', { class: 'label' }, label),
        h(
            'div',
            { class: 'row' },
            h('input', {
                type: 'range',
                min,
                max,
                step: opts.step || 1,
                value,
                disabled: opts.disabled,
                oninput: e => {
                    out.textContent = e.target.value;
                    onChange(e.target.value);
                }
            }),
            out
        )
    );
}

export function Button(text, onClick, opts) {
    opts = opts || {};
    return h(
        'button',
        { class: (opts.primary ? 'primary ' : '') + (opts.class || ''), disabled: opts.disabled, title: opts.title, onclick: onClick },
        text
    );
}

// a list with a selected item and add / delete buttons (the left pane of the reference's multi-item tabs:
// reference data, functions, outputs, rules, batches)
export function ItemList(items, selectedIndex, labelOf, onSelect, onAdd, onDelete, opts) {
    opts = opts || {};
    return h(
        'div',
        { class: 'itemlist' },
        h(
            'div',
            { class: 'row' },
            onAdd ? opts.addMenu || Button('+ Add', onAdd, { disabled: opts.addDisabled }) : null,
            onDelete && items.length
                ? Button('Delete', () => onDelete(selectedIndex), { disabled: opts.deleteDisabled || !opts.canDelete(selectedIndex) })
                : null
        ),
        h(
            'ul',
            null,
            items.map((it, i) =>
                h(
                    'li',
                    {
                        class: (i === selectedIndex ? 'on' : '') + (opts.isValid && !opts.isValid(it) ? ' invalid' : ''),
                        onclick: () => onSelect(i)
                    },
                    labelOf(it, i)
                )
            )
        )
    );
}

export function Table(columns, rows, opts) {
    opts = opts || {};
    return h(
        'table',
        { class: 'grid' + (opts.compact ? ' compact' : '') },
        h('thead', null, h('tr', null, columns.map(c => h('th', null, c.name)))),
        h(
            'tbody',
            null,
            rows.map(r =>
                h(
                    'tr',
                    { onclick: opts.onRowClick ? () => opts.onRowClick(r) : null },
                    columns.map(c => h('td', null, c.render ? c.render(r) : r[c.key] === undefined ? '' : String(r[c.key])))
                )
            )
        )
    );
}

// rerenderable component root: state changes call update(), which rebuilds the children
export function component(render) {
    const root = h('div', { class: 'component' });
    const update = () => mount(root, render(update));
    update();
    return { root, update };
}
