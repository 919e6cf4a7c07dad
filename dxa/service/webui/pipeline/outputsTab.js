// Outputs tab (datax-pipeline flowDefinition/components/output/*: outputSettingsContent and the per-sink
// blobSinkerSettings, cosmosdbSinkerSettings, eventHubSinkerSettings, sqlSinkerSettings, localSinkerSettings,
// metricSinkerSettings). A sink's id is what the query's `OUTPUT <table> TO <id>` names.
import { h } from '../common/dom.js';
import { TextField, Dropdown, Toggle, ItemList, StatementBox, Button, functionEnabled } from '../common/components.js';
import * as Models from './models.js';
import * as V from './validation.js';

const idError = v => (V.isNumberAndStringOnly(v || '') ? null : 'letters and digits only');

function settings(o, ui) {
    const p = o.properties;
    const f = (label, key, opts) => TextField(label, p[key], v => { p[key] = v; ui.touch(); }, opts);
    const secret = { type: 'password' };
    switch (o.type) {
        case 'metric':
            return StatementBox('i', 'The built-in metric sink: OUTPUT tables sent here are charted on the flow\'s ' +
                'metrics dashboard (each row needs MetricName, Metric and EventTime / uts columns).');
        case 'blob':
            return h('div', null,
                f('Storage account connection string (kept in the secret store)', 'connectionString', secret),
                f('Container', 'containerName', { validate: idError }),
                f('Blob prefix (folder under the container)', 'blobPrefix'),
                f('Partition format (yyyy/MM/dd/HH)', 'blobPartitionFormat'),
                Dropdown('Format', Models.sinkerFormatTypes, p.format, v => { p.format = v; ui.touch(); }),
                Dropdown('Compression (gzip is done on the GPU)', Models.sinkerCompressionTypes, p.compressionType, v => { p.compressionType = v; ui.touch(); }));
        case 'local':
            return h('div', null,
                f('Folder', 'folder'),
                f('Prefix', 'blobPrefix'),
                f('Partition format (yyyy/MM/dd/HH)', 'blobPartitionFormat'),
                Dropdown('Format', Models.sinkerFormatTypes, p.format, v => { p.format = v; ui.touch(); }),
                Dropdown('Compression', Models.sinkerCompressionTypes, p.compressionType, v => { p.compressionType = v; ui.touch(); }));
        case 'cosmosdb':
            return h('div', null,
                f('Cosmos DB connection string (AccountEndpoint=...;AccountKey=...)', 'connectionString', secret),
                f('Database', 'db', { validate: idError }),
                f('Collection', 'collection', { validate: idError }));
        case 'eventhub':
            return h('div', null,
                f('Event Hub connection string (with EntityPath)', 'connectionString', secret),
                Dropdown('Format', Models.sinkerFormatTypes, p.format, v => { p.format = v; ui.touch(); }),
                Dropdown('Compression', Models.sinkerCompressionTypes, p.compressionType, v => { p.compressionType = v; ui.touch(); }));
        case 'sql':
            return h('div', null,
                f('SQL Server connection string (Server=...;Database=...;User ID=...;Password=...)', 'connectionString', secret),
                f('Database (optional if in the connection string)', 'databaseName'),
                f('Table', 'tableName'),
                Dropdown('Write mode', Models.sqlWriteModes, p.writeMode, v => { p.writeMode = v; ui.touch(); }),
                Toggle('Use bulk insert (TDS bulk load)', p.useBulkInsert, v => { p.useBulkInsert = v; ui.touch(); }));
        case 'httppost':
            return h('div', null, f('Endpoint URL', 'endpoint'), f('Filter (optional SQL condition)', 'filter'));
        case 'console':
            return h('div', null, f('Rows printed per batch', 'maxRows'));
        default:
            return h('div', { class: 'errtext' }, `unknown sink type ${o.type}`);
    }
}

export function OutputsTab(flow, ui) {
    const items = flow.outputs;
    let sel = Math.min(ui.selected.outputs || 0, Math.max(0, items.length - 1));
    const disabled = !functionEnabled('addOutputSinkButtonEnabled');
    const typeSel = h('select', { disabled }, Models.sinkerTypes.map(t => h('option', { value: t.key }, t.name)));
    const add = h('div', { class: 'row' }, typeSel, Button('+ Add', () => {
        const o = Models.defaultSinker(typeSel.value);
        o.id = typeSel.value + (items.length + 1);
        items.push(o);
        ui.selected.outputs = items.length - 1;
        ui.touch();
        ui.update();
    }, { disabled }));
    const o = items[sel];
    return h(
        'div',
        { class: 'cols' },
        ItemList(items, sel, x => `${x.id || '(new)'} · ${x.type}`, i => { ui.selected.outputs = i; ui.update(); },
            () => null, i => { items.splice(i, 1); ui.touch(); ui.update(); }, {
                isValid: V.isSinkerComplete,
                addMenu: add,
                deleteDisabled: !functionEnabled('deleteOutputSinkButtonEnabled'),
                canDelete: i => items[i] && items[i].type !== 'metric'
            }),
        h('div', { class: 'grow' },
            o
                ? h('div', null,
                    TextField('Sink id (used in OUTPUT ... TO <id>)', o.id, v => { o.id = v; ui.touch(); },
                        { validate: idError, disabled: o.type === 'metric' }),
                    h('div', { class: 'muted' }, 'Type: ' + ((Models.sinkerTypes.find(t => t.key === o.type) || { name: o.type }).name)),
                    settings(o, ui))
                : h('div', { class: 'muted' }, 'No outputs.'))
    );
}
